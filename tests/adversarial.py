"""TEST INFRASTRUCTURE: config 3's in-place adversarial mutation (tools/adversarial_batch.py) with the
C oracle as the forger of the mixed-order class, so tests do not depend on libsodium's group API."""
from adversarial_batch import CLASSES, inject as _inject  # noqa: F401


def inject(blob, off, pks, frac, seed, oracle):
    """Mutates copies of blob/pks; returns (blob, pks, idx, classes)."""
    return _inject(blob, off, pks, frac, seed, forger=oracle)
