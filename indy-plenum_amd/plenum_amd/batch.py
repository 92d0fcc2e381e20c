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
def active(cache, engine=None, answers=None):
    """Run per-request logic against a batch's verdicts. ``answers`` (optional): {id(req_data):
    (req_data, authenticator, identifiers)} for requests whose whole authenticate() outcome the
    batch already knows (the wire plan's device-finished requests)."""
    _stack().append((cache, engine, answers))
    try:
        yield cache
    finally:
        _stack().pop()


def answer(authnr, req_data):
    """The identifiers ``authnr.authenticate(req_data)`` returns, when the active batch computed
    them for this very request object and authenticator (every signature verified on the device,
    signers resolved exactly as authenticate resolves them); else None."""
    s = _stack()
    if not s or not s[-1][2]:
        return None
    a = s[-1][2].get(id(req_data))
    if a is None or a[0] is not req_data or a[1] is not authnr:
        return None
    return list(a[2])


def verdict(pk, sm):
    """crypto_sign_open verdict for one pair: from the active batch cache, else one launch."""
    s = _stack()
    engine = None
    if s:
        cache, engine, _ = s[-1]
        v = cache.get(pk, sm)
        if v is not None:
            return v
    if engine is None:  # one launch of one pair, no arrays built around it
        return _native.verify_one(pk, sm)
    return bool(verify_pairs([(pk, sm)], engine)[0])
