"""The C ABI boundary: libplenum_verify.so loads without a GPU, exports exactly what
include/plenum_verify.h declares (and what the ctypes shim binds), refuses compute loudly when no
GPU is present, and its CPU-side host-prep entry points (base58, DidVerifier key resolution) agree
with the oracle restatement and the reference's golden vectors."""
import ctypes
import json
import os
import random
import re

import numpy as np
import pytest

from oracle.base58_ref import b58decode as ref_b58decode, b58encode as ref_b58encode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "plenum_verify.h")
TEST_HEADER = os.path.join(ROOT, "include", "plenum_verify_test.h")


def header_functions(path=None):
    paths = [path] if path else [HEADER, TEST_HEADER]
    out = set()
    for p in paths:
        text = re.sub(r"/\*.*?\*/", "", open(p).read(), flags=re.S)
        out |= set(re.findall(r"\b(pv_[a-z0-9_]+)\s*\(", text))
    return out


@pytest.fixture(scope="module")
def native():
    from plenum_amd import _native
    return _native


def test_library_exports_every_declared_symbol(native):
    L = native.lib()
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert declared == set(native.SIGNATURES), declared ^ set(native.SIGNATURES)
    assert L.pv_abi_version() == native.PV_ABI_VERSION


def L_stamps_absent(native):
    """The product build compiles no clock stamps (PV_CLOCK_PROBE is a diagnostic build only)."""
    return native.lib().pv_test_clock_stamps(None, 0) == 0


def test_test_hooks_outside_the_product_header(native):
    """The fault-injection hook is declared only in the test header, and refuses to act unless
    PV_ENABLE_TEST_HOOKS=1 is set (a production caller must not be able to arm it)."""
    assert "pv_test_inject" not in header_functions(HEADER)
    assert header_functions(TEST_HEADER) == {"pv_test_inject", "pv_test_clock_stamps"}
    assert L_stamps_absent(native)
    L = native.lib()
    old = os.environ.pop("PV_ENABLE_TEST_HOOKS", None)
    try:
        assert L.pv_test_inject(native.PV_INJECT_STAGE, 0, 1) == native.PV_ERR_ARG
        assert b"disabled" in L.pv_last_error()
        os.environ["PV_ENABLE_TEST_HOOKS"] = "1"
        assert L.pv_test_inject(native.PV_INJECT_STAGE, 0, 0) == native.PV_OK
    finally:
        if old is None:
            os.environ.pop("PV_ENABLE_TEST_HOOKS", None)
        else:
            os.environ["PV_ENABLE_TEST_HOOKS"] = old


def test_no_gpu_fails_loudly(native):
    L = native.lib()
    if L.pv_device_count() > 0:
        pytest.skip("a GPU is visible")
    assert L.pv_init(0) < 0
    with pytest.raises(native.NativeUnavailable):
        native.verify_sm_batch(np.zeros(64, np.uint8), np.array([0, 64], np.uint64), np.zeros((1, 32), np.uint8))
    # the product authentication path has no CPU fallback either
    from plenum_amd.nacl_wrappers import Verifier
    with pytest.raises(native.NativeUnavailable):
        Verifier(bytes(32)).verify(bytes(64), b"msg")


def test_fastcall_binding_matches_ctypes_entry(native):
    """The CPython binding (plenum_amd/_fastcall.c: buffer protocol, GIL released) calls the same
    pv_verify_batch the ctypes path binds: without an initialised device both return the library's
    not-initialised code; inconsistent sizes are refused before the call."""
    fc = native._fastcall()
    if not fc:
        pytest.skip("_fastcall not built (make -C indy-plenum_amd)")
    L = native.lib()
    if L.pv_device_count() > 0:
        pytest.skip("a GPU is visible")
    blob, off = np.zeros(64, np.uint8), np.array([0, 64], np.uint64)
    pks, bits = np.zeros((1, 32), np.uint8), np.zeros(1, np.uint8)
    rc_c = L.pv_verify_batch(native._ptr(blob), native._ptr(off), 1, native._ptr(pks), native._ptr(bits))
    assert rc_c != native.PV_OK and fc.verify(blob, off, pks, bits) == rc_c
    for bad in ((blob, np.array([0, 65], np.uint64), pks, bits),           # record past the blob
                (blob, off, np.zeros(16, np.uint8), bits),                  # short key array
                (blob, np.array([0], np.uint64), pks, bits),                # no request
                (blob, off, pks, np.zeros(0, np.uint8))):                   # no verdict byte
        with pytest.raises(ValueError):
            fc.verify(*bad)
    with pytest.raises((TypeError, BufferError)):
        fc.verify(blob, off, pks, bytes(1))                                 # read-only verdict buffer
    # the one-pair call (the unbatched drop-in): the same entry point and return code
    assert fc.verify_one(bytes(32), bytes(64)) == rc_c
    with pytest.raises(ValueError):
        fc.verify_one(bytes(31), bytes(64))                                 # short key


def test_b58decode_batch_vs_restatement():
    from plenum_amd.base58 import b58decode_many, b58encode
    rng = random.Random(4)
    alphabet = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"
    vals = ["", "1", "111", "1112", "2", "z" * 90, "  ", "abc \t\n", "0abc", "1l1", "ab c", "é"]
    for _ in range(500):
        vals.append("".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 100))))
    for _ in range(50):
        data = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 70)))
        data = b"\0" * rng.randrange(0, 4) + data
        vals.append(ref_b58encode(data).decode())
    got = b58decode_many(vals)
    for v, g in zip(vals, got):
        try:
            want = ref_b58decode(v)
        except Exception as ex:
            assert isinstance(g, Exception) and type(g) is type(ex) and str(g) == str(ex), (v, g, ex)
            continue
        assert g == want, v
    for _ in range(200):
        data = b"\0" * rng.randrange(0, 3) + bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 64)))
        assert b58encode(data) == ref_b58encode(data)


def test_resolve_verkeys_matches_reference_golden(native):
    """pv_resolve_verkeys (batched DidVerifier resolution) against the reference's outcomes."""
    with open(os.path.join(ROOT, "tests", "golden", "didverifier.json")) as f:
        cases = json.load(f)
    usable = [c for c in cases if all(isinstance(x, str) or x is None for x in (c["verkey"], c["identifier"]))
              and all((x or "").isascii() and (x or "") == (x or "").rstrip() for x in (c["verkey"], c["identifier"]))]
    n = len(usable)
    idr = [(c["identifier"] or "").encode() for c in usable]
    vk = [(c["verkey"] or "").encode() for c in usable]
    has_vk = np.array([c["verkey"] is not None for c in usable], np.uint8)

    def pack(strs):
        off = np.zeros(len(strs) + 1, np.uint64)
        np.cumsum([len(s) for s in strs], out=off[1:])
        buf = np.frombuffer(b"".join(strs) or b"\0", np.uint8)
        return buf, off

    ib, io = pack(idr)
    vb, vo = pack(vk)
    pk = np.zeros((n, 32), np.uint8)
    st = np.zeros(n, np.uint8)
    L = native.lib()
    assert L.pv_resolve_verkeys(ib.ctypes.data, io.ctypes.data, vb.ctypes.data, vo.ctypes.data, has_vk.ctypes.data,
                                n, pk.ctypes.data, st.ctypes.data) == 0
    for i, c in enumerate(usable):
        out = c["out"]
        if "exc" in out:
            want = {"ValueError": (1, 4), "InvalidKey": (2,)}[out["exc"]]
            assert st[i] in want, (c, st[i])
            if st[i] == 1:
                assert out["msg"] == "'verkey' should be a non-empty string"
        elif out["value"]["raw"] is None:
            assert st[i] == 3, c
        else:
            assert st[i] == 0, c
            assert pk[i].tobytes().hex() == out["value"]["raw"], c
