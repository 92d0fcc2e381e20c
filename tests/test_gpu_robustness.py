"""GPU robustness of the C ABI beyond the parity classes:
  * the 220 committed libsodium verdict vectors (tests/golden/verdicts.json) on the HIP engine, every
    arithmetic path;
  * long messages up to Plenum's MSG_LEN_LIMIT (128 KiB, stp_core/config.py:27) mixed into the same
    waves as ~300 B records (SHA-512 loops of 10^2-10^3 blocks beside 3-block ones), every path;
  * two different batches enqueued back-to-back on two caller streams (pv_verify_batch_device's
    workspace hand-over), and host-buffer + ingress calls from two threads at once."""
import json
import os
import threading

import numpy as np
import pytest

from vectors import VectorGen, pack

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
MSG_LEN_LIMIT = 128 * 1024  # stp_core/config.py:27


@pytest.fixture(scope="module")
def nat():
    from plenum_amd import _native
    _native.ensure_device()
    yield _native
    _native.set_path(_native.PV_PATH_AUTO)


def _paths(nat):
    return [(name, getattr(nat, "PV_PATH_" + name.upper())) for name in nat.PATH_NAMES]


def _sodium_verdicts(sodium, cases):
    return np.array([sodium.sign_open_ok(sm, pk) for sm, pk in cases], dtype=bool)


def test_golden_verdict_vectors_on_gpu(nat):
    with open(os.path.join(HERE, "golden", "verdicts.json")) as f:
        vec = json.load(f)
    cases = [(bytes.fromhex(c["sm"]), bytes.fromhex(c["pk"])) for c in vec]
    want = np.array([c["ok"] for c in vec], dtype=bool)
    blob, off, pks = pack(cases)
    for name, mode in _paths(nat):
        nat.set_path(mode)
        got = nat.verify_sm_batch(blob, off, pks)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (name, [vec[i]["cls"] for i in bad[:5]])
    nat.set_path(nat.PV_PATH_AUTO)


def test_verify_one_golden_vectors(nat, sodium):
    """The unbatched drop-in's one-pair call (_native.verify_one: _fastcall.verify_one, no arrays) on
    the 220 committed libsodium vectors, an empty message and a 128 KiB one, and through
    nacl_wrappers.Verifier outside any batch: libsodium's verdicts; a short key raises."""
    from plenum_amd.nacl_wrappers import Verifier
    with open(os.path.join(HERE, "golden", "verdicts.json")) as f:
        vec = json.load(f)
    for c in vec:
        assert nat.verify_one(bytes.fromhex(c["pk"]), bytes.fromhex(c["sm"])) == c["ok"], c["cls"]
    pk, sk = sodium.seed_keypair(b"\x07" * 32)
    for m in (b"", bytes(range(256)) * 512):
        sm = sodium.sign_detached(m, sk) + m
        assert nat.verify_one(pk, sm) is True
        assert Verifier(pk).verify(sm[:64], m) is True
        bad = bytearray(sm)
        bad[-1 if m else 0] ^= 1
        assert nat.verify_one(pk, bytes(bad)) is False
        assert Verifier(pk).verify(bytes(bad[:64]), bytes(bad[64:])) is False
    with pytest.raises(ValueError):
        nat.verify_one(pk[:31], sm)


def test_long_messages_mixed_with_short(nat, sodium, oracle):
    g = VectorGen(sodium, oracle, seed=21)
    rng = np.random.default_rng(21)
    cases = []
    for i in range(192):
        if i % 24 == 5:  # a long record inside a wave of short ones
            size = int(rng.choice([16 * 1024, 40 * 1024 + 3, 100 * 1024 + 1, MSG_LEN_LIMIT]))
            m = rng.bytes(size)
            cases.append(g.valid(m))
        else:
            cases.append(g.valid(rng.bytes(int(rng.integers(280, 320)))))
    # corrupt a few long and short ones (message tail, signature)
    for i in (5, 29, 77):
        sm = bytearray(cases[i][0])
        sm[-1] ^= 1
        cases[i] = (bytes(sm), cases[i][1])
    for i in (6, 100):
        sm = bytearray(cases[i][0])
        sm[40] ^= 2
        cases[i] = (bytes(sm), cases[i][1])
    blob, off, pks = pack(cases)
    want = _sodium_verdicts(sodium, cases)
    assert want.sum() == len(cases) - 5
    for name, mode in _paths(nat):
        nat.set_path(mode)
        got = nat.verify_sm_batch(blob, off, pks)
        assert np.array_equal(got, want), (name, np.nonzero(got != want)[0][:10])
    nat.set_path(nat.PV_PATH_AUTO)


class _Dev:
    def __init__(self, nat, blob, off, pks):
        import ctypes
        self.nat, self.L = nat, nat.lib()
        self.ptrs = []
        self.n = len(off) - 1
        self.blob = self.put(np.concatenate([blob, np.zeros(nat.PV_BLOB_SLACK, np.uint8)]))
        self.off = self.put(np.ascontiguousarray(off, np.uint64))
        self.pk = self.put(np.ascontiguousarray(pks, np.uint8))
        self.words = (self.n + 63) // 64
        self.ver = self.alloc(self.words * 8)
        self.ctypes = ctypes

    def alloc(self, nbytes):
        import ctypes
        p = ctypes.c_void_p()
        self.nat.check(self.L.pv_dev_alloc(ctypes.byref(p), nbytes), "pv_dev_alloc")
        self.ptrs.append(p)
        return p

    def put(self, a):
        p = self.alloc(a.nbytes)
        self.nat.check(self.L.pv_memcpy_h2d(p, a.ctypes.data, a.nbytes), "pv_memcpy_h2d")
        return p

    def verdicts(self):
        out = np.zeros(self.words, np.uint64)
        self.nat.check(self.L.pv_memcpy_d2h(out.ctypes.data, self.ver, out.nbytes), "pv_memcpy_d2h")
        return np.unpackbits(out.view(np.uint8), bitorder="little")[:self.n].astype(bool)

    def free(self):
        for p in self.ptrs:
            self.L.pv_dev_free(p)


def test_two_caller_streams_back_to_back(nat, sodium, oracle):
    """Two different batches, each large enough for the keyed comb path's shared workspace, enqueued
    on two caller streams with no synchronisation between them; then a small one on a third."""
    import ctypes
    import nym_workload
    nat.set_path(nat.PV_PATH_AUTO)
    a = nym_workload.generate(0, 50000, workers=8)
    b = nym_workload.generate(900000, 40000, workers=8)
    bb = b[0].copy()
    bad_b = np.arange(7, 40000, 997)
    for i in bad_b:
        bb[int(b[1][i]) + 80] ^= 0x10
    g = VectorGen(sodium, oracle, seed=31)
    small = g.batch(300, adversarial_frac=0.3)
    c = pack(small)
    L = nat.lib()
    streams = [ctypes.c_void_p() for _ in range(3)]
    for s in streams:
        nat.check(L.pv_stream_create(ctypes.byref(s)), "pv_stream_create")
    devs = [_Dev(nat, a[0], a[1], a[2]), _Dev(nat, bb, b[1], b[2]), _Dev(nat, *c)]
    try:
        for rep in range(3):
            for d, s in zip(devs, streams):
                nat.check(L.pv_verify_batch_device(d.blob, d.off, d.n, d.pk, d.ver, s), "pv_verify_batch_device")
            for s in streams:
                nat.check(L.pv_stream_sync(s), "pv_stream_sync")
            assert devs[0].verdicts().all()
            want_b = np.ones(40000, bool)
            want_b[bad_b] = False
            assert np.array_equal(devs[1].verdicts(), want_b)
            assert np.array_equal(devs[2].verdicts(), _sodium_verdicts(sodium, small))
    finally:
        for d in devs:
            d.free()
        for s in streams:
            L.pv_stream_destroy(s)


def test_two_threads_host_and_ingress(nat, sodium, oracle):
    """verify_sm_batch and ingress_verify_arrays from two threads at once (ctypes releases the GIL),
    several rounds; every result matches libsodium / the sequential call."""
    import nym_workload
    from plenum_amd import _native
    g = VectorGen(sodium, oracle, seed=41)
    cases = g.batch(2000, adversarial_frac=0.05)
    blob, off, pks = pack(cases)
    want = _sodium_verdicts(sodium, cases)
    # ingress: NYM requests over the wire form (b58 signatures, signer strings)
    n = 3000
    rb, ro, rp, wblob, woff, sblob, soff = nym_workload.generate_wire(0, n, workers=8)
    pool = nym_workload._pool()
    ib, io = _native._blob([p["did"].encode() for p in pool])
    vb, vo = _native._blob([p["abbr"].encode() for p in pool])
    vp = np.ones(len(pool), np.uint8)
    mblob = np.concatenate([rb[int(ro[i]) + 64:int(ro[i + 1])] for i in range(n)])
    moff = np.zeros(n + 1, np.uint64)
    np.cumsum(np.diff(ro) - 64, out=moff[1:])
    args = (sblob, soff, mblob, moff, np.arange(n, dtype=np.uint32), (np.arange(n) % len(pool)).astype(np.uint32),
            ib, io, vb, vo, vp)
    st0, v0 = _native.ingress_verify_arrays(*args)
    assert (st0 == 0).all() and v0.all()
    errors = []

    def host_loop():
        try:
            for _ in range(6):
                got = _native.verify_sm_batch(blob, off, pks)
                if not np.array_equal(got, want):
                    errors.append(("host", np.nonzero(got != want)[0][:5]))
        except Exception as e:  # pragma: no cover
            errors.append(("host", repr(e)))

    def ingress_loop():
        try:
            for _ in range(6):
                st, v = _native.ingress_verify_arrays(*args)
                if not ((st == 0).all() and v.all()):
                    errors.append(("ingress", int((~v).sum())))
        except Exception as e:  # pragma: no cover
            errors.append(("ingress", repr(e)))

    ts = [threading.Thread(target=host_loop), threading.Thread(target=ingress_loop)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors


_BCOMB16_SCRIPT = r"""
import json, os, sys
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "indy-plenum_amd"), os.path.join(root, "tests"), os.path.join(root, "tools")]
import numpy as np
import nym_workload, adversarial_batch
from oracle.oracle import cpu_verdicts
from plenum_amd import _native
blob, off, pks = nym_workload.generate(0, 300000, workers=8)
blob, pks, idx, labels = adversarial_batch.inject(blob, off, pks, 0.02, seed=9)
want = cpu_verdicts(blob, off, pks)
_native.ensure_device(0)
out = {}
for name in ("auto", "comb", "straus"):
    _native.set_path(getattr(_native, "PV_PATH_" + name.upper()))
    got = _native.verify_sm_batch(blob, off, pks)
    out[name] = {"mismatches": int((got != want).sum()), "split": list(_native.last_split())}
out["rejected"] = int((~want).sum())
print(json.dumps(out))
"""


def test_wide_comb_fallback_radix16_bit_exact(sodium):
    """pv_init's fallback when the 10.7 GB wide fixed-base comb cannot be allocated (forced here with
    PV_FORCE_BCOMB16): [S]B from the radix-65536 comb on the keyed and Straus paths. A fresh process
    (the radix is chosen once per pv_init) verifies 300k NYM requests with 2 % adversarial records on
    every throughput path; verdicts must equal libsodium's."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PV_FORCE_BCOMB16="1")
    p = subprocess.run([sys.executable, "-c", _BCOMB16_SCRIPT, root], env=env, capture_output=True, text=True,
                       timeout=170)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["rejected"] > 5000
    for name in ("auto", "comb", "straus"):
        assert res[name]["mismatches"] == 0, (name, res)
    assert res["auto"]["split"][1] >= 1024  # the signers took the comb path
