"""In-place adversarial mutation of a large packed batch: BASELINE configs[2] ("1M requests with ~2 %
adversarial signatures"), SURVEY.md §8c (iv) classes.

Every class keeps the record length, so the packed blob/offsets stay valid: bit flips in R/S/A/M,
S + L, S in {L, L+1, 2^253-1, 2^256-1}, small-order R / A (with and without bit 255), non-canonical
A, off-curve A, non-canonical R, mixed-order keys A + T8 with an honest signature over the
record's own message, and mixed-order R' = rB + [j]T8 with S = r + k a under a prime-order key
(never accepted) or under A + T8 (accepted iff [j]T8 = -[k]T8, about one in eight). The forger for the mixed-order class is libsodium 1.0.18 itself
(crypto_scalarmult_ed25519_base_noclamp, crypto_core_ed25519_add, the reference's own native
dependency) plus hashlib's SHA-512, so bench.py can build the batch without the test oracle; the
tests pass the C oracle's forger instead (tests/adversarial.py). Seeded and deterministic.
"""
import ctypes
import hashlib

import numpy as np

P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493
# the 7 libsodium small-order encodings (ge25519_has_small_order)
BLACKLIST = [
    bytes(32),
    bytes([1]) + bytes(31),
    bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"),
    bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"),
    (P - 1).to_bytes(32, "little"),
    P.to_bytes(32, "little"),
    (P + 1).to_bytes(32, "little"),
]
ORDER8 = BLACKLIST[2]

CLASSES = ("flip_R", "flip_S", "flip_A", "flip_M", "S_plus_L", "S_big", "R_blacklist", "A_blacklist",
           "A_noncanonical", "A_offcurve", "R_noncanonical", "mixed_order_A", "mixed_order_R", "mixed_order_AR")


class SodiumForger:
    """Raw-scalar Ed25519 signing with libsodium's group operations: what no honest signer can
    produce (a key with a small-order component), needed for the mixed-order class."""

    def __init__(self, lib=None):
        if lib is None:
            import nym_workload
            lib = nym_workload.sodium()
        self.lib = lib
        for fn in ("crypto_scalarmult_ed25519_base_noclamp", "crypto_core_ed25519_add"):
            getattr(lib, fn).restype = ctypes.c_int

    def scalarmult_base(self, s: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        if self.lib.crypto_scalarmult_ed25519_base_noclamp(out, s) != 0:
            raise ValueError("scalar is zero")
        return out.raw

    def point_add(self, p: bytes, q: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        if self.lib.crypto_core_ed25519_add(out, p, q) != 0:
            raise ValueError("not a point")
        return out.raw

    def sign_raw(self, r: bytes, a: bytes, A_enc: bytes, msg: bytes) -> bytes:
        """R = [r]B, S = r + H(R || A || M) a mod L (RFC 8032 verification equation)."""
        R = self.scalarmult_base(r)
        k = int.from_bytes(hashlib.sha512(R + A_enc + msg).digest(), "little") % L
        S = (int.from_bytes(r, "little") + k * int.from_bytes(a, "little")) % L
        return R + S.to_bytes(32, "little")


def _offcurve_ys(rng, k):
    d = (-121665 * pow(121666, P - 2, P)) % P
    ys = []
    while len(ys) < k:
        y = int(rng.integers(1, 2 ** 62)) * int(rng.integers(1, 2 ** 62)) % P
        u = (y * y - 1) % P
        v = (d * y * y + 1) % P
        t = u * pow(v, P - 2, P) % P
        if t and pow(t, (P - 1) // 2, P) != 1:
            ys.append(y)
    return ys


def inject(blob, off, pks, frac, seed, forger=None):
    """Mutates copies of blob/pks; returns (blob, pks, idx, classes). forger: an object with
    scalarmult_base / point_add / sign_raw (default: SodiumForger)."""
    forger = forger or SodiumForger()
    rng = np.random.default_rng(seed)
    blob = blob.copy()
    pks = pks.copy()
    n = len(off) - 1
    k = max(len(CLASSES), int(n * frac))
    idx = np.sort(rng.choice(n, size=k, replace=False))
    labels = []
    offc = _offcurve_ys(rng, 64)
    t8 = [ORDER8]  # [j]T8, j = 1..7
    for _ in range(6):
        t8.append(forger.point_add(t8[-1], ORDER8))
    for j, i in enumerate(idx):
        cls = CLASSES[j % len(CLASSES)]
        labels.append(cls)
        o0, o1 = int(off[i]), int(off[i + 1])
        sig = blob[o0:o0 + 64]
        if cls == "flip_R":
            sig[int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif cls == "flip_S":
            sig[32 + int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif cls == "flip_A":
            pks[i, int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif cls == "flip_M":
            if o1 > o0 + 64:
                blob[int(rng.integers(o0 + 64, o1))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif cls == "S_plus_L":
            s = int.from_bytes(sig[32:].tobytes(), "little") + L
            sig[32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        elif cls == "S_big":
            s = [L, L + 1, 2 ** 253 - 1, 2 ** 256 - 1][j % 4]
            sig[32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        elif cls == "R_blacklist":
            b = bytearray(BLACKLIST[j % 7])
            b[31] |= 0x80 * (j % 2)
            sig[:32] = np.frombuffer(bytes(b), np.uint8)
        elif cls == "A_blacklist":
            b = bytearray(BLACKLIST[j % 7])
            b[31] |= 0x80 * (j % 2)
            pks[i] = np.frombuffer(bytes(b), np.uint8)
        elif cls == "A_noncanonical":
            b = bytearray((P + j % 19).to_bytes(32, "little"))
            b[31] |= 0x80 * (j % 2)
            pks[i] = np.frombuffer(bytes(b), np.uint8)
        elif cls == "A_offcurve":
            pks[i] = np.frombuffer(offc[j % len(offc)].to_bytes(32, "little"), np.uint8)
        elif cls == "R_noncanonical":
            y = P + j % 19
            b = bytearray(y.to_bytes(32, "little"))
            b[31] |= int(sig[31]) & 0x80
            sig[:32] = np.frombuffer(bytes(b), np.uint8)
        elif cls == "mixed_order_A":
            a = int(rng.integers(1, 2 ** 62)) * int(rng.integers(1, 2 ** 62)) % L or 1
            A = forger.scalarmult_base(a.to_bytes(32, "little"))
            A2 = forger.point_add(A, ORDER8)
            r = (int(rng.integers(1, 2 ** 62)) * 7919 % L or 1).to_bytes(32, "little")
            msg = blob[o0 + 64:o1].tobytes()
            s2 = forger.sign_raw(r, a.to_bytes(32, "little"), A2, msg)
            sig[:] = np.frombuffer(s2, np.uint8)
            pks[i] = np.frombuffer(A2, np.uint8)
        elif cls in ("mixed_order_R", "mixed_order_AR"):
            a = int(rng.integers(1, 2 ** 62)) * int(rng.integers(1, 2 ** 62)) % L or 1
            A = forger.scalarmult_base(a.to_bytes(32, "little"))
            if cls == "mixed_order_AR":
                A = forger.point_add(A, ORDER8)
            r = int(rng.integers(1, 2 ** 62)) * 7919 % L or 1
            R = forger.point_add(forger.scalarmult_base(r.to_bytes(32, "little")), t8[j % 7])
            msg = blob[o0 + 64:o1].tobytes()
            k = int.from_bytes(hashlib.sha512(R + A + msg).digest(), "little") % L
            sig[:] = np.frombuffer(R + ((r + k * a) % L).to_bytes(32, "little"), np.uint8)
            pks[i] = np.frombuffer(A, np.uint8)
    return blob, pks, idx, labels


def tamper(blob, off, k, seed):
    """Flips one message byte in k seeded records of a valid batch (the headline's must-reject
    records): returns (blob copy, sorted indices). A flipped message byte changes k = H(R||A||M), so
    libsodium rejects exactly these records."""
    rng = np.random.default_rng(seed)
    n = len(off) - 1
    idx = np.sort(rng.choice(n, size=min(k, n), replace=False))
    blob = blob.copy()
    for i in idx:
        o0, o1 = int(off[i]), int(off[i + 1])
        if o1 > o0 + 64:
            blob[int(rng.integers(o0 + 64, o1))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    return blob, idx
