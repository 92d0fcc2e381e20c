"""Verdict plumbing between the batched GPU launch and the per-request Python logic.

``authenticate_batch`` (client_authn / req_authenticator) first collects every (public key,
signature||message) pair the batch will need, verifies them in ONE engine launch, and then runs
the unchanged per-request logic inside ``active(cache)``; ``verdict()`` answers from the cache
and only launches the engine for pairs the plan did not foresee (or outside a batch).
This keeps the reference's exact control flow — dict-order loops, threshold short-circuits,
exception order, one ``authenticate`` call per request (plenum/test/node_request/
test_propagate/test_no_reauth.py:11-23) — while the signature arithmetic is batched.
"""
import threading
from contextlib import contextmanager

import numpy as np

from . import _native

_tls = threading.local()


class VerdictCache:
    def __init__(self):
        self._v = {}
        self.hits = 0
        self.misses = 0

    def fill(self, pairs, engine=None):
        """pairs: list of (pk32 bytes, sm bytes); verifies the ones not cached yet in one launch."""
        todo = [p for p in dict.fromkeys(pairs) if p not in self._v]
        if not todo:
            return
        verdicts = verify_pairs(todo, engine)
        for p, ok in zip(todo, verdicts):
            self._v[p] = bool(ok)

    def get(self, pk, sm):
        v = self._v.get((pk, sm))
        if v is None:
            self.misses += 1
        else:
            self.hits += 1
        return v

    def __len__(self):
        return len(self._v)


def pack_pairs(pairs):
    n = len(pairs)
    lens = np.fromiter((len(sm) for _, sm in pairs), dtype=np.uint64, count=n)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    blob = np.frombuffer(b"".join(sm for _, sm in pairs), dtype=np.uint8)
    pks = np.frombuffer(b"".join(pk for pk, _ in pairs), dtype=np.uint8).reshape(n, 32)
    return blob, off, pks


def verify_pairs(pairs, engine=None):
    """Verdicts for [(pk, sm)] through ``engine`` (a callable (blob, off, pks) -> bool array);
    the default engine is the HIP library."""
    if not pairs:
        return np.zeros(0, dtype=bool)
    blob, off, pks = pack_pairs(pairs)
    fn = engine or _native.verify_sm_batch
    return np.asarray(fn(blob, off, pks), dtype=bool)


def _stack():
    s = getattr(_tls, "stack", None)
    if s is None:
        s = _tls.stack = []
    return s


@contextmanager
def active(cache, engine=None):
    _stack().append((cache, engine))
    try:
        yield cache
    finally:
        _stack().pop()


def verdict(pk, sm):
    """crypto_sign_open verdict for one pair: from the active batch cache, else one launch."""
    s = _stack()
    engine = None
    if s:
        cache, engine = s[-1]
        v = cache.get(pk, sm)
        if v is not None:
            return v
    return bool(verify_pairs([(pk, sm)], engine)[0])
