"""ctypes binding to libsodium 1.0.18 — the native library the reference actually calls.

ORACLE / TEST INFRASTRUCTURE ONLY. The reference reaches libsodium through libnacl 1.6.1
(setup.py:107-108): ``stp_core/crypto/nacl_wrappers.py:108`` calls
``libnacl.crypto_sign_open(sm, pk)``, which calls libsodium ``crypto_sign_open`` and raises
``ValueError`` on a nonzero return. libnacl is not installed in this image; libsodium 1.0.18 is
(``/opt/conda/lib/libsodium.so.23``, the same version as the reference's pinned ``libsodium23``
package). This module reproduces that call exactly, plus the signing/keypair
functions used to generate fixtures, and a multi-threaded C-loop timing harness is in
``cpu_baseline.c``.
"""
import ctypes
import os

_CANDIDATES = ("/opt/conda/lib/libsodium.so.23", "/usr/lib/x86_64-linux-gnu/libsodium.so.23")


def find_libsodium():
    for p in _CANDIDATES:
        if os.path.exists(p):
            return p
    return None


class LibSodium:
    def __init__(self, path=None):
        path = path or find_libsodium()
        if path is None:
            raise OSError("libsodium.so.23 not found in %r" % (_CANDIDATES,))
        self.path = path
        self.lib = ctypes.CDLL(path)
        if self.lib.sodium_init() < 0:
            raise OSError("sodium_init failed")
        self.lib.sodium_version_string.restype = ctypes.c_char_p
        self.version = self.lib.sodium_version_string().decode()

    def seed_keypair(self, seed: bytes):
        assert len(seed) == 32
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        if self.lib.crypto_sign_seed_keypair(pk, sk, seed) != 0:
            raise ValueError("keypair failed")
        return pk.raw, sk.raw

    def sign_detached(self, msg: bytes, sk: bytes) -> bytes:
        sig = ctypes.create_string_buffer(64)
        siglen = ctypes.c_ulonglong()
        if self.lib.crypto_sign_detached(sig, ctypes.byref(siglen), msg, ctypes.c_ulonglong(len(msg)), sk):
            raise ValueError("sign failed")
        return sig.raw

    def sign_open_ok(self, sm: bytes, pk: bytes) -> bool:
        """libnacl.crypto_sign_open semantics (True = it would return the message)."""
        if len(pk) != 32:
            raise ValueError("Invalid public key")
        out = ctypes.create_string_buffer(max(len(sm), 1))
        outlen = ctypes.c_ulonglong()
        return self.lib.crypto_sign_open(out, ctypes.byref(outlen), sm, ctypes.c_ulonglong(len(sm)), pk) == 0
