"""GPU parity at BASELINE.json's sizes (configs 2-4), through the C ABI:
  config 2  1M single-signature NYM requests: every verdict 1 (valid by construction)
  config 3  1M requests with ~2 % adversarial: verdicts bit-exact vs libsodium 1.0.18 on every record
  config 4  multi-signature (3 endorsers, authenticate_multi semantics): the device verdicts of the
            expanded (request, signer) records vs libsodium, and the per-request reduction vs the
            reference's loop rules
plus the product authenticate path on the real engine against the reference's golden outcomes."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def native():
    from plenum_amd import _native
    _native.ensure_device()
    return _native


@pytest.fixture(scope="module")
def nym1m():
    import nym_workload
    return nym_workload.generate(0, 1 << 20)


def test_config2_1M_valid(native, nym1m):
    blob, off, pks = nym1m
    got = native.verify_sm_batch(blob, off, pks)
    assert got.all()


@pytest.fixture(scope="module")
def adv1m(nym1m, oracle):
    """configs[2]: the 1M batch with 2 % adversarial records, and libsodium's verdicts."""
    from adversarial import inject
    from oracle.oracle import cpu_verdicts
    blob, off, pks = nym1m
    blob2, pks2, idx, labels = inject(blob, off, pks, 0.02, seed=3, oracle=oracle)
    return blob2, off, pks2, idx, cpu_verdicts(blob2, off, pks2)


def test_config3_1M_adversarial_bit_exact(native, adv1m, oracle):
    blob2, off, pks2, idx, want = adv1m
    # both arithmetic paths: the per-request Straus path and the keyed comb path (~10k distinct
    # keys here: the 1,024 signers plus every mutated key). Device-resident, the batch is ONE launch
    # chunk (the fused comb kernel for AUTO / COMB); from host buffers it runs as pipelined
    # sub-batches of 262,144 requests that share the first one's comb tables
    from bench import DeviceBatch, bits
    db = DeviceBatch(blob2, off, pks2)
    try:
        for path in (native.PV_PATH_STRAUS, native.PV_PATH_COMB, native.PV_PATH_AUTO):
            native.set_path(path)
            db.verify()
            got = bits(db.verdict_words(), len(want))
            split = native.last_split()
            native.set_path(native.PV_PATH_AUTO)
            assert np.array_equal(got, want), (path, np.nonzero(got != want)[0][:10])
            if path == native.PV_PATH_AUTO:
                # the 1,024 signers get comb tables; the adversarial one-request keys take the Straus
                # path in the same launch
                # (plus the few adversarial keys that recur: blacklisted / non-canonical encodings)
                assert 1024 <= split[1] < 1200 and split[0] > split[1], split
                assert len(got) - 30000 < split[2] < len(got), split
    finally:
        db.free()
    for path in (native.PV_PATH_STRAUS, native.PV_PATH_AUTO):
        native.set_path(path)
        got = native.verify_sm_batch(blob2, off, pks2)
        native.set_path(native.PV_PATH_AUTO)
        assert np.array_equal(got, want), ("host", path, np.nonzero(got != want)[0][:10])
    # the untouched 98 % are valid and the mutated records are (almost all) rejected
    mask = np.ones(len(got), bool)
    mask[idx] = False
    assert got[mask].all()
    assert (~got[idx]).sum() > 0.9 * len(idx)
    # the oracle agrees on the adversarial records too
    sub = idx[:600]
    o = np.array([oracle.sign_open_ok(blob2[off[i]:off[i + 1]].tobytes(), pks2[i].tobytes()) for i in sub])
    assert np.array_equal(o, got[sub])


def test_config3_1M_cached_signers_bit_exact(native, adv1m):
    """configs[2] with the 1,024 signers in the node-side key cache (pv_key_cache_put): a cached
    signer's requests read the cache's affine rows in the comb kernels (D = 2 Z1, no Z1 Z2 product;
    comb.h pv_comb_row_to_affine), the adversarial keys are not cached and get tables built in the
    launch or go Straus. Forced COMB and AUTO, device-resident (one 1M chunk: the fused kernel) and from
    host buffers (pipelined sub-batches on the cached tables), every verdict equal to libsodium's."""
    import nym_workload
    from bench import DeviceBatch, bits
    blob2, off, pks2, idx, want = adv1m
    kc = native.KeyCache
    kc.configure(2048)
    db = DeviceBatch(blob2, off, pks2)
    try:
        kc.put([p["vk"] for p in nym_workload._pool()])
        assert kc.stats()[0] == 1024
        for path in (native.PV_PATH_COMB, native.PV_PATH_AUTO):
            native.set_path(path)
            db.verify()
            got = bits(db.verdict_words(), len(want))
            split = native.last_split()
            assert np.array_equal(got, want), (path, np.nonzero(got != want)[0][:10])
            assert split[1] >= 1024, split  # every cached signer is a comb key
            got = native.verify_sm_batch(blob2, off, pks2)
            native.set_path(native.PV_PATH_AUTO)
            assert np.array_equal(got, want), ("host", path, np.nonzero(got != want)[0][:10])
    finally:
        native.set_path(native.PV_PATH_AUTO)
        db.free()
        kc.configure(0)


def test_config4_multisig(native, sodium):
    """configs[3] at its stated size: 1,048,576 requests with 3 signatures each (author + 2
    endorsers over the same payload), expanded to 3,145,728 (request, signer) records = 3 launch
    chunks; 1 % of the records carry a flipped R/S bit at seeded positions among the 3. Device
    verdicts bit-exact against libsodium on every record, and the authenticate_multi reduction
    (threshold None: all must verify, client_authn.py:84-118) equal to the expected one."""
    import bench
    import nym_workload
    from oracle.oracle import cpu_verdicts
    n_req, k = 1 << 20, 3
    blob, off, pk, bad = nym_workload.generate_multisig(0, n_req, k, bad_frac=0.01, seed=4)
    assert bad.sum() == int(n_req * k * 0.01) and bad.any(axis=1).sum() > 30000
    got = native.verify_sm_batch(blob, off, pk).reshape(n_req, k)
    want = cpu_verdicts(blob, off, pk).reshape(n_req, k)
    assert np.array_equal(got, want), np.argwhere(got != want)[:10]
    assert np.array_equal(~got, bad)
    acc, correct = bench.multisig_reduce(got)
    assert acc.sum() == n_req - bad.any(axis=1).sum()
    assert np.array_equal(correct, k - bad.sum(axis=1))
    # the device-resident leg the bench times: same records, same verdicts
    native.set_path(native.PV_PATH_AUTO)
    from bench import DeviceBatch, bits
    db = DeviceBatch(blob, off, pk)
    try:
        db.verify()  # the copy-back is stream-ordered after the launch: no pv_sync
        assert np.array_equal(bits(db.verdict_words(), n_req * k).reshape(n_req, k), want)
    finally:
        db.free()


def test_product_authn_golden_on_gpu(native):
    from plenum_amd.client_authn import CoreAuthNr
    from plenum_amd.req_authenticator import ReqAuthenticator
    from plenum_amd.state_utils import DictState
    with open(os.path.join(HERE, "golden", "authn.json")) as f:
        data = json.load(f)

    def outcome(fn):
        try:
            r = fn()
            return {"list": r} if isinstance(r, list) else {"value": r}
        except Exception as ex:
            return {"exc": type(ex).__name__, "msg": str(ex)}

    def mk():
        a = CoreAuthNr(["1", "101"], ["105"], ["action"], state=DictState(data["state_nyms"]))
        for idr, vk in data["clients"].items():
            a.addIdr(idr, vk)
        return a

    for c in data["cases"]:  # sequential: one single-request launch per signature
        req = json.loads(json.dumps(c["req"]))
        a = mk()
        fn = (lambda: a.authenticate(req, **c["kw"])) if c["kind"] == "authenticate" else \
            (lambda: a.authenticate_multi(req, **c["kw"]))
        assert outcome(fn) == c["out"], c
    cases = [c for c in data["cases"] if c["kind"] == "authenticate" and not c["kw"]]
    res = mk().authenticate_batch([json.loads(json.dumps(c["req"])) for c in cases])
    for c, r in zip(cases, res):
        got = {"exc": type(r).__name__, "msg": str(r)} if isinstance(r, Exception) else {"list": r}
        assert got == c["out"], c
    with open(os.path.join(HERE, "golden", "reqauth.json")) as f:
        ra_data = json.load(f)
    seq = ra_data["seqs"][0]
    ra = ReqAuthenticator()
    core = CoreAuthNr(["1", "101"], ["105"], ["action"], state=DictState({}))
    for idr, vk in ra_data["clients"].items():
        core.addIdr(idr, vk)
    ra.register_authenticator(core)
    res = ra.authenticate_batch([(json.loads(json.dumps(r)), k) for r, k in seq["items"]])
    got = [({"exc": type(x).__name__, "msg": str(x)} if isinstance(x, Exception) else {"set": sorted(x)}) for x in res]
    assert got == seq["out"]


def test_rccl_allgather_single_rank(native):
    from plenum_amd.sharding import RcclGather, verify_sharded
    from vectors import pack
    import nym_workload
    blob, off, pks = nym_workload.generate(5000, 3000, workers=1)
    g = RcclGather(1, 0, RcclGather.unique_id())
    assert g.comm_count() == (1, 0)  # what RCCL itself reports for the one-rank communicator
    got = verify_sharded(blob, off, pks, 0, 1, native.verify_sm_batch, g)
    assert got.all() and len(got) == 3000


def test_smoke_entry():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ge", os.path.join(os.path.dirname(HERE), "__graft_entry__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m.smoke()


def test_two_chunks_every_path(native, nym1m):
    """More requests than one launch chunk (2^20): the second chunk is small, so AUTO takes the
    Straus path there while the first chunk goes keyed-comb; forced paths cover both chunks.
    A few corrupted records in each chunk must be rejected on every path."""
    blob, off, pks = nym1m
    extra = 100000
    blob2 = np.concatenate([blob, blob[:int(off[extra])]])
    off2 = np.concatenate([off, off[1:extra + 1] + off[-1]])
    pks2 = np.concatenate([pks, pks[:extra]])
    n = len(off2) - 1
    bad = np.array([5, 777777, (1 << 20) + 3, n - 1])
    for i in bad:
        blob2[int(off2[i]) + 70] ^= 1  # a message byte
    want = np.ones(n, bool)
    want[bad] = False
    for path in (native.PV_PATH_AUTO, native.PV_PATH_COMB, native.PV_PATH_STRAUS):
        native.set_path(path)
        got = native.verify_sm_batch(blob2, off2, pks2)
        native.set_path(native.PV_PATH_AUTO)
        assert np.array_equal(got, want), (path, np.nonzero(got != want)[0][:10])


def test_config5_shard_8M(native, nym1m):
    """Config 5 (64M requests over 8 GPUs) as one GPU sees it: its 8M-request shard, 8 launch
    chunks, each chunk deduplicating its keys and taking the comb path. Tiled from the 1M NYM set;
    the 24 records corrupted across the chunks must be exactly the rejected ones."""
    blob, off, pks = nym1m
    reps = 8
    n1, total = len(off) - 1, int(off[-1])
    blob8 = np.tile(blob, reps)
    off8 = np.concatenate([off[:-1] + np.uint64(r * total) for r in range(reps)]
                          + [np.array([reps * total], np.uint64)]).astype(np.uint64)
    pks8 = np.tile(pks, (reps, 1))
    n = n1 * reps
    bad = np.sort(np.random.default_rng(5).choice(n, 24, replace=False))
    bad[0], bad[-1] = 0, n - 1
    for i in bad:
        blob8[int(off8[i]) + 70] ^= 0x20  # a message byte
    want = np.ones(n, bool)
    want[bad] = False
    got = native.verify_sm_batch(blob8, off8, pks8)
    assert len(got) == n
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


def _split_batch(sodium, n_signed, n_single, seed):
    """n_signed NYM requests from the 1,024-signer pool (n_signed / 1,024 per key) plus n_single
    requests that each carry their own key, shuffled, with ~1 % of records corrupted."""
    import nym_workload
    rng = np.random.default_rng(seed)
    recs, keys = [], []
    if n_signed:
        blob, off, pks = nym_workload.generate(7000, n_signed, workers=8)
        recs = [blob[off[i]:off[i + 1]].tobytes() for i in range(n_signed)]
        keys = [pks[i].tobytes() for i in range(n_signed)]
    for j in range(n_single):
        pk, sk = sodium.seed_keypair(rng.bytes(32))
        m = rng.bytes(int(rng.integers(0, 320)))
        recs.append(sodium.sign_detached(m, sk) + m)
        keys.append(pk)
    perm = rng.permutation(len(recs))
    recs = [bytearray(recs[i]) for i in perm]
    keys = [keys[i] for i in perm]
    bad = rng.choice(len(recs), len(recs) // 100, replace=False)
    for i in bad:
        recs[i][int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
    off2 = np.zeros(len(recs) + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=off2[1:])
    return (np.frombuffer(b"".join(bytes(r) for r in recs), np.uint8), off2,
            np.frombuffer(b"".join(keys), np.uint8).reshape(-1, 32))


def test_split_paths_in_one_launch(native, sodium):
    """Frequent signers and one-off keys in one chunk: AUTO gives tables to the 1,024 frequent keys
    (60 requests each) and verifies the 20,000 one-off requests on the Straus path; forced COMB
    gives tables to the first 16,384 keys only (the capacity) and the rest go Straus; every path
    bit-exact against libsodium."""
    from oracle.oracle import cpu_verdicts
    blob, off, pks = _split_batch(sodium, 61440, 20000, seed=11)
    n = len(off) - 1
    want = cpu_verdicts(blob, off, pks)
    assert 0 < (~want).sum() < n // 50
    for path in (native.PV_PATH_AUTO, native.PV_PATH_COMB, native.PV_PATH_STRAUS):
        native.set_path(path)
        got = native.verify_sm_batch(blob, off, pks)
        split = native.last_split()
        native.set_path(native.PV_PATH_AUTO)
        assert np.array_equal(got, want), (path, np.nonzero(got != want)[0][:10])
        if path == native.PV_PATH_AUTO:
            assert split == (21024, 1024, 61440), split
        elif path == native.PV_PATH_COMB:
            assert split[0] == 21024 and split[1] == 16384 and 16384 < split[2] < n, split


def test_split_all_keys_distinct(native, sodium):
    """A chunk big enough for dedup in which no key repeats: AUTO builds no table and every request
    goes through the Straus path in slot order."""
    from oracle.oracle import cpu_verdicts
    blob, off, pks = _split_batch(sodium, 0, 40000, seed=12)
    want = cpu_verdicts(blob, off, pks)
    got = native.verify_sm_batch(blob, off, pks)
    assert native.last_split() == (40000, 0, 0)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


def test_medium_chunks_all_comb_or_split(native, sodium):
    """AUTO at medium sizes: a 20k chunk with few distinct keys (1,024 signers + 600 one-off keys)
    makes every key a comb key, one-request keys included; a 20k chunk with more than 2,048
    distinct keys keeps the >= 48-requests rule (the 1,024 signers' ~19 requests each stay Straus
    side). Both bit-exact against libsodium, as are the forced paths."""
    from oracle.oracle import cpu_verdicts
    for n_signed, n_single, want_all in ((19456, 600, True), (12288, 4000, False)):
        blob, off, pks = _split_batch(sodium, n_signed, n_single, seed=13 + n_single)
        n = len(off) - 1
        want = cpu_verdicts(blob, off, pks)
        got = native.verify_sm_batch(blob, off, pks)
        keys_all, comb_keys, comb_req = native.last_split()
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
        assert keys_all == 1024 + n_single, keys_all
        if want_all:
            assert (comb_keys, comb_req) == (keys_all, n), (comb_keys, comb_req)
        else:
            assert comb_keys == 0 and comb_req == 0, (comb_keys, comb_req)
        for path in (native.PV_PATH_COMB, native.PV_PATH_STRAUS):
            native.set_path(path)
            got = native.verify_sm_batch(blob, off, pks)
            native.set_path(native.PV_PATH_AUTO)
            assert np.array_equal(got, want), (path, np.nonzero(got != want)[0][:10])


def test_dedup_hot_keys(native):
    """Key skew far beyond the bench's ~1,000 requests per signer, in a chunk large enough for the
    dedup's seed pass (> 65,536 requests): 120k requests of one signer, 60k of another and 20k
    spread over the 1,024-signer pool, shuffled, ~0.1 % corrupted. Every key's requests must land in
    one contiguous slot range (the per-key counters are split 8 ways and re-joined by the assign
    kernel), so AUTO (all keys comb here) and forced COMB must equal libsodium bit for bit."""
    import nym_workload
    from oracle.oracle import cpu_verdicts
    blob, off, pks = nym_workload.generate(0, 4096)
    rng = np.random.default_rng(21)
    src = np.concatenate([np.zeros(120000, np.int64), np.ones(60000, np.int64),
                          rng.integers(2, 4096, 20000)])
    src = src[rng.permutation(len(src))]
    lens = (off[1:] - off[:-1]).astype(np.int64)[src]
    off2 = np.zeros(len(src) + 1, np.uint64)
    np.cumsum(lens, out=off2[1:])
    blob2 = np.concatenate([blob[int(off[s]):int(off[s + 1])] for s in src])
    pks2 = np.ascontiguousarray(pks[src])
    n = len(src)
    for i in rng.choice(n, 200, replace=False):
        blob2[int(off2[i]) + int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
    want = cpu_verdicts(blob2, off2, pks2)
    assert 150 < (~want).sum() <= 200
    for path in (native.PV_PATH_AUTO, native.PV_PATH_COMB):
        native.set_path(path)
        got = native.verify_sm_batch(blob2, off2, pks2)
        split = native.last_split()
        native.set_path(native.PV_PATH_AUTO)
        assert np.array_equal(got, want), (path, np.nonzero(got != want)[0][:10])
        assert split == (1024, 1024, n), (path, split)


def test_medium_host_batch_path_hint(native, sodium):
    """Host batches between 2,048 and 4,096 requests: with >= 3 requests per key AUTO takes the keyed
    path (the host counts the keys, pv_keyed_hint), with one-off keys the latency path; both
    bit-exact against libsodium, as are the forced paths."""
    from oracle.oracle import cpu_verdicts
    for n_signed, n_single, want_path in ((4096, 0, native.PV_PATH_COMB), (3072, 0, native.PV_PATH_COMB),
                                          (2048, 0, native.PV_PATH_LATENCY),
                                          (0, 3000, native.PV_PATH_LATENCY)):
        blob, off, pks = _split_batch(sodium, n_signed, n_single, seed=31 + n_signed)
        want = cpu_verdicts(blob, off, pks)
        got = native.verify_sm_batch(blob, off, pks)
        path, _ = native.last_path()
        assert path == want_path, (n_signed, n_single, path)
        assert np.array_equal(got, want), (n_signed, n_single, np.nonzero(got != want)[0][:10])
        for forced in (native.PV_PATH_LATENCY, native.PV_PATH_COMB):
            native.set_path(forced)
            got = native.verify_sm_batch(blob, off, pks)
            native.set_path(native.PV_PATH_AUTO)
            assert np.array_equal(got, want), (forced, np.nonzero(got != want)[0][:10])


def test_medium_device_batch_path_choice(native, sodium):
    """The device-buffer twin of test_medium_host_batch_path_hint: pv_verify_batch_device cannot
    count keys on the host, so for 2,049..4,096 requests AUTO runs the dedup kernels and lets the
    scan pick (>= 3 requests per key: keyed; else the latency kernel runs and the keyed kernels exit
    at once). Same paths and bit-exact verdicts as the host-buffer call; verdict words that held
    stale bits before the call are fully rewritten on both outcomes."""
    from bench import DeviceBatch, bits
    from oracle.oracle import cpu_verdicts
    native.set_path(native.PV_PATH_AUTO)
    for n_signed, n_single, want_path in ((4096, 0, native.PV_PATH_COMB), (3072, 0, native.PV_PATH_COMB),
                                          (2048, 8, native.PV_PATH_LATENCY),
                                          (0, 3000, native.PV_PATH_LATENCY), (0, 4096, native.PV_PATH_LATENCY)):
        blob, off, pks = _split_batch(sodium, n_signed, n_single, seed=41 + n_signed + n_single)
        n = len(off) - 1
        want = cpu_verdicts(blob, off, pks)
        db = DeviceBatch(blob, off, pks)
        try:
            stale = np.full(db.words, 0xA5A5A5A5A5A5A5A5, np.uint64)
            native.check(native.lib().pv_memcpy_h2d(db.d_verdict, stale.ctypes.data, stale.nbytes), "h2d")
            db.verify()
            native.check(native.lib().pv_sync(), "pv_sync")
            got = bits(db.verdict_words(), n)
            path, _ = native.last_path()
            assert path == want_path, (n_signed, n_single, path)
            assert np.array_equal(got, want), (n_signed, n_single, np.nonzero(got != want)[0][:10])
            # the next launch on the same workspace (the other outcome) still sees a clean table
            db.verify()
            native.check(native.lib().pv_sync(), "pv_sync")
            assert np.array_equal(bits(db.verdict_words(), n), want)
        finally:
            db.free()
