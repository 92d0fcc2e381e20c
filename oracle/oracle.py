"""ctypes loader for the C oracle (ed25519_oracle.c). ORACLE / TEST INFRASTRUCTURE ONLY."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


class Oracle:
    def __init__(self):
        if not os.path.exists(_LIB):
            build()
        self.lib = ctypes.CDLL(_LIB)
        self.lib.oracle_sign_open.restype = ctypes.c_int
        self.lib.oracle_sign_open.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        self.lib.oracle_sign_open_batch.restype = None
        self.lib.oracle_sign_open_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]

    def sign_open_ok(self, sm: bytes, pk: bytes) -> bool:
        assert len(pk) == 32
        return self.lib.oracle_sign_open(sm, ctypes.c_size_t(len(sm)), pk) == 0

    def verify_batch(self, blob: np.ndarray, off: np.ndarray, pk: np.ndarray, lo=0, hi=None) -> np.ndarray:
        n = len(off) - 1
        hi = n if hi is None else hi
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        pk = np.ascontiguousarray(pk, dtype=np.uint8)
        out = np.zeros(n, dtype=np.uint8)
        self.lib.oracle_sign_open_batch(blob.ctypes.data, off.ctypes.data, pk.ctypes.data,
                                        ctypes.c_uint64(lo), ctypes.c_uint64(hi), out.ctypes.data)
        return out[lo:hi]

    def sc_reduce64(self, x: bytes) -> bytes:
        r = ctypes.create_string_buffer(32)
        self.lib.oracle_sc_reduce64(r, x)
        return r.raw

    def scalarmult_base(self, s: bytes) -> bytes:
        r = ctypes.create_string_buffer(32)
        self.lib.oracle_scalarmult_base(r, s)
        return r.raw

    def point_add(self, p: bytes, q: bytes):
        r = ctypes.create_string_buffer(32)
        if self.lib.oracle_point_add(r, p, q) != 0:
            return None
        return r.raw

    def sign_raw(self, r: bytes, a: bytes, A_enc: bytes, msg: bytes) -> bytes:
        sig = ctypes.create_string_buffer(64)
        self.lib.oracle_sign_raw(sig, r, a, A_enc, msg, ctypes.c_size_t(len(msg)))
        return sig.raw

    def sha512(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.lib.oracle_sha512_3(out, data, ctypes.c_size_t(len(data)), None, ctypes.c_size_t(0), None,
                                 ctypes.c_size_t(0))
        return out.raw


def cpu_verdicts(blob, off, pks, threads=None):
    """Per-record crypto_sign_open verdicts from libsodium 1.0.18 (the oracle if it is absent), threaded."""
    import numpy as np
    from oracle.libsodium_ref import find_libsodium
    o = Oracle()
    fn = o.lib.cpu_verdicts
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    path = find_libsodium()
    threads = threads or min(16, len(os.sched_getaffinity(0)))
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    pks = np.ascontiguousarray(pks, dtype=np.uint8)
    n = len(off) - 1
    out = np.zeros(n, dtype=np.uint8)
    rc = fn((path or "").encode(), 1 if path else 0, blob.ctypes.data, off.ctypes.data, pks.ctypes.data, n, threads,
            out.ctypes.data)
    if rc != 0:
        raise OSError("cpu_verdicts failed")
    return out.astype(bool)
