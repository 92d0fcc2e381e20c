"""base58 (Bitcoin alphabet) with the semantics of PyPI ``base58`` 2.x ``b58decode``/``b58encode``
— the package the reference imports at plenum/server/client_authn.py:7 and
plenum/common/verifier.py:4 (unpinned in setup.py:98-99).

str-level rules are applied here exactly as the package does (``str.rstrip()`` strips Unicode
whitespace, then the text must encode as ASCII, else ``UnicodeEncodeError``, a ``ValueError``);
the bignum conversion runs in libplenum_verify (C++ ``pv_b58decode_batch`` / ``pv_b58encode``),
batched for the authenticate_batch path.
"""
import ctypes

import numpy as np

from . import _native

ALPHABET = b"123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"
_VALID = frozenset(ALPHABET)


def _scrub(v):
    v = v.rstrip()  # None -> AttributeError, exactly as base58.b58decode(None)
    if isinstance(v, str):
        v = v.encode('ascii')
    return bytes(v)


def _invalid_char(v: bytes):
    body = v.lstrip(b"1")
    for c in body:
        if c not in _VALID:
            return ValueError("Invalid character {!r}".format(chr(c)))
    return None


def b58decode_many(values, max_len=512):
    """Decode a list of str/bytes. Returns a list whose items are bytes or the exception that
    ``base58.b58decode`` would raise for that input."""
    scrubbed, results = [], [None] * len(values)
    for i, v in enumerate(values):
        try:
            scrubbed.append(_scrub(v))
        except Exception as ex:  # UnicodeEncodeError, AttributeError (None), TypeError
            results[i] = ex
            scrubbed.append(b"")
    n = len(values)
    if n == 0:
        return results
    chars = b"".join(scrubbed)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([len(s) for s in scrubbed], out=off[1:])
    stride = max(1, max(len(s) for s in scrubbed), max_len)
    out = np.zeros((n, stride), dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.uint8)
    buf = np.frombuffer(chars, dtype=np.uint8) if chars else np.zeros(1, np.uint8)
    _native.check(_native.lib().pv_b58decode_batch(
        buf.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p), n,
        out.ctypes.data_as(ctypes.c_void_p), stride, out_len.ctypes.data_as(ctypes.c_void_p),
        status.ctypes.data_as(ctypes.c_void_p)), "pv_b58decode_batch")
    for i in range(n):
        if results[i] is not None:
            continue
        if status[i] == 0:
            results[i] = out[i, :out_len[i]].tobytes()
        elif status[i] == 1:
            results[i] = _invalid_char(scrubbed[i]) or ValueError("Invalid character")
        else:  # cannot happen: stride >= input length >= output length
            results[i] = ValueError("base58 output too long")
    return results


def b58decode(v):
    """One value (the per-signature calls of the sequential path): the same C++ conversion as
    b58decode_many, called on the bytes directly, without the batch's array packing."""
    s = _scrub(v)
    n = len(s)
    out = ctypes.create_string_buffer(max(n, 1))
    out_len, status = ctypes.c_uint32(), ctypes.c_uint8()
    _native.check(_native.lib().pv_b58decode_batch(s, (ctypes.c_uint64 * 2)(0, n), 1, out, max(n, 1),
                                                   ctypes.byref(out_len), ctypes.byref(status)),
                  "pv_b58decode_batch")
    if status.value == 0:
        return out.raw[:out_len.value]
    if status.value == 1:
        raise _invalid_char(s) or ValueError("Invalid character")
    raise ValueError("base58 output too long")


def b58encode(v) -> bytes:
    if isinstance(v, str):
        v = v.encode('ascii')
    data = bytes(v)
    L = _native.lib()
    cap = 2 * len(data) + 2
    out = ctypes.create_string_buffer(cap)
    n = L.pv_b58encode(data, len(data), out, cap)
    return out.raw[:n]
