"""GPU parity of the device ingress front end (pv_ingress_verify): base58 decode
of every signature, DidVerifier key resolution per signer, device-side sm assembly, verification.

Expected values come from the checkers, never from the product: base58 from oracle/base58_ref.py
(the restatement pinned by the reference's KAT), key resolution from the reference's own
DidVerifier outcomes (tests/golden/didverifier.json) and from pv_resolve_verkeys (host C++, pinned
against the same goldens in test_abi.py), verdicts from libsodium 1.0.18 crypto_sign_open on
b58decode(sig) || M."""
import json
import os

import numpy as np
import pytest

from oracle.base58_ref import b58decode as ref_b58decode, b58encode as ref_b58encode

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def native():
    from plenum_amd import _native
    _native.ensure_device()
    return _native


def host_key_status(native, idrs, vks):
    """pv_resolve_verkeys on the host (golden-pinned) -> (status, pk) per signer."""
    n = len(idrs)
    ib, io = native._blob(idrs)
    vb, vo = native._blob([v if v is not None else b"" for v in vks])
    has = np.array([v is not None for v in vks], np.uint8)
    pk = np.zeros((n, 32), np.uint8)
    st = np.zeros(n, np.uint8)
    native.check(native.lib().pv_resolve_verkeys(ib.ctypes.data, io.ctypes.data, vb.ctypes.data, vo.ctypes.data,
                                                 has.ctypes.data, n, pk.ctypes.data, st.ctypes.data),
                 "pv_resolve_verkeys")
    return st, pk


def expected(sodium, native, sigs, msgs, msg_idx, signer_idx, idrs, vks):
    kst, kpk = host_key_status(native, idrs, vks)
    status, verdict = [], []
    for sig, mi, si in zip(sigs, msg_idx, signer_idx):
        try:
            raw = ref_b58decode(sig)
        except ValueError:
            status.append(1)
            verdict.append(False)
            continue
        if len(raw) > 96:
            status.append(2)
            verdict.append(False)
            continue
        if kst[si]:
            status.append(16 + int(kst[si]))
            verdict.append(False)
            continue
        status.append(0)
        verdict.append(sodium.sign_open_ok(raw + msgs[mi], kpk[si].tobytes()))
    return np.array(status, np.uint8), np.array(verdict, bool)


def signer_forms(sodium, rng, count):
    """Signers in every verkey form the reference accepts: DidSigner (DID + '~' abbreviated
    verkey), cryptonym (identifier = full key, no verkey), full verkey, hex verkey."""
    out = []
    for i in range(count):
        pk, sk = sodium.seed_keypair(rng.bytes(32))
        form = i % 4
        if form == 0:
            idr, vk = ref_b58encode(pk[:16]), b"~" + ref_b58encode(pk[16:])
        elif form == 1:
            idr, vk = ref_b58encode(pk), None
        elif form == 2:
            idr, vk = ref_b58encode(pk[:16]), ref_b58encode(pk)
        else:
            idr, vk = ref_b58encode(pk[:16]), ref_b58encode(pk.hex().encode())
        out.append((idr, vk, sk))
    return out


def signature_variant(kind, sig, rng):
    """Encodings of one signature covering every b58decode / sm-assembly rule."""
    if kind == 1:
        return ref_b58encode(sig[:63])  # shifts the signature / message split point
    if kind == 2:
        return ref_b58encode(sig + b"\x07")
    if kind == 3:
        return ref_b58encode(sig)[:-1] + b"0"  # character outside the alphabet
    if kind == 4:
        return b""
    if kind == 5:
        return ref_b58encode(b"\0\0" + sig)  # leading '1's
    if kind == 6:
        return ref_b58encode(sig) + b" \t\n"  # trailing ASCII whitespace
    if kind == 7:
        return ref_b58encode(rng.bytes(97))  # decodes to more than 96 bytes
    if kind == 8:
        return ref_b58encode(sig[:1] + bytes([sig[1] ^ 4]) + sig[2:])  # one bit changed
    if kind == 9:
        return b"1" * 100  # 100 zero bytes
    if kind == 10:
        return b"\xc3\xa9" + ref_b58encode(sig)  # non-ASCII byte
    return ref_b58encode(sig)


# signer table rows whose key resolution fails in each documented way (statuses 17..20)
ODD_SIGNERS = [
    (b"99BgFBg35BehzfSADV5nM4", None), (b"99BgFBg35BehzfSADV5nM4", b""), (b"0OIl", b"~8zH9ZSyZTFPGJ4ZPL5Rvxx"),
    (b"99BgFBg35BehzfSADV5nM4", b"~0OIl"), (b"99BgFBg35BehzfSADV5nM4", b"~2"), (b"", None), (b"", b""),
    (b"", b"   "), (b"99BgFBg35BehzfSADV5nM4", b"~"), (b"  ", b"~" + ref_b58encode(bytes(range(1, 33)))),
    (b"1111111111111111", b"~1111111111111111"), (b"FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF", None)]


def test_signature_and_key_variants(native, sodium):
    rng = np.random.default_rng(21)
    signers = signer_forms(sodium, rng, 16)
    good = len(signers)
    idrs = [s[0] for s in signers] + [b[0] for b in ODD_SIGNERS]
    vks = [s[1] for s in signers] + [b[1] for b in ODD_SIGNERS]
    msgs = [rng.bytes(int(rng.integers(0, 400))) for _ in range(40)]
    sigs, msg_idx, signer_idx = [], [], []
    for j in range(600):
        mi = int(rng.integers(0, len(msgs)))
        si = int(rng.integers(0, good)) if j % 5 else int(rng.integers(0, len(idrs)))
        sig = sodium.sign_detached(msgs[mi], signers[si][2]) if si < good else rng.bytes(64)
        sigs.append(signature_variant(j % 13, sig, rng))
        msg_idx.append(mi)
        signer_idx.append(si)
    st, v = native.ingress_verify(sigs, msgs, msg_idx, signer_idx, idrs, vks)
    want_st, want_v = expected(sodium, native, sigs, msgs, msg_idx, signer_idx, idrs, vks)
    diff = np.nonzero((st != want_st) | (v != want_v))[0]
    assert len(diff) == 0, [(i, sigs[i], signer_idx[i], st[i], want_st[i], v[i], want_v[i]) for i in diff[:6]]
    assert want_v.sum() > 150 and (want_st == 0).sum() > 300
    assert set(int(x) for x in want_st) >= {0, 1, 2, 17, 18, 19, 20}


def test_key_status_matches_reference_golden(native):
    """Device key resolution vs the reference's DidVerifier outcomes (every ASCII golden case)."""
    with open(os.path.join(ROOT, "tests", "golden", "didverifier.json")) as f:
        cases = json.load(f)
    usable = [c for c in cases if all(isinstance(x, str) or x is None for x in (c["verkey"], c["identifier"]))
              and all((x or "").isascii() and (x or "") == (x or "").rstrip() for x in (c["verkey"], c["identifier"]))]
    idrs = [(c["identifier"] or "").encode() for c in usable]
    vks = [c["verkey"].encode() if c["verkey"] is not None else None for c in usable]
    n = len(usable)
    sig = ref_b58encode(b"\x01" * 64)  # decodes, so the status is 16 + the key status
    st, _ = native.ingress_verify([sig] * n, [b"m" * 10], [0] * n, list(range(n)), idrs, vks)
    for i, c in enumerate(usable):
        out = c["out"]
        k = int(st[i]) - 16 if st[i] else 0
        if "exc" in out:
            assert k in {"ValueError": (1, 4), "InvalidKey": (2,)}[out["exc"]], (c, st[i])
        elif out["value"]["raw"] is None:
            assert k == 3, c
        else:
            assert k == 0, c


def test_many_requests_multi_signature(native, sodium):
    """Three endorser signatures over one M per request (authenticate_multi), 64 signers in every
    verkey form, 49,152 verifications over many scan tiles; every verdict True except the flipped
    ones."""
    rng = np.random.default_rng(5)
    signers = signer_forms(sodium, rng, 64)
    idrs = [s[0] for s in signers]
    vks = [s[1] for s in signers]
    nreq = 1 << 14
    msgs = [b"identifier:%d|operation:dest:x|reqId:%d" % (i % 97, i) + rng.bytes(int(rng.integers(200, 300)))
            for i in range(nreq)]
    sigs, mi, si, flipped = [], [], [], []
    for r in range(nreq):
        for k in range(3):
            s = (3 * r + k) % 64
            sig = sodium.sign_detached(msgs[r], signers[s][2])
            t = (r * 3 + k) % 101 == 0
            if t:
                sig = bytes([sig[0] ^ 1]) + sig[1:]
            sigs.append(ref_b58encode(sig))
            mi.append(r)
            si.append(s)
            flipped.append(t)
    st, v = native.ingress_verify(sigs, msgs, mi, si, idrs, vks)
    assert (st == 0).all()
    assert np.array_equal(v, ~np.array(flipped))


def test_out_of_range_indices_are_errors(native):
    with pytest.raises(native.NativeError):
        native.ingress_verify([b"2"], [b"m"], [5], [0], [b"99BgFBg35BehzfSADV5nM4"], [None])
    with pytest.raises(native.NativeError):
        native.ingress_verify([b"2"], [b"m"], [0], [3], [b"99BgFBg35BehzfSADV5nM4"], [None])
