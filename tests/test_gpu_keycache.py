"""GPU: the node-side key cache (pv_key_cache_*). A cached key is verified on the latency path with
32 comb-table additions instead of 252 doublings; verdicts must stay exactly libsodium's, including
keys that fail libsodium's key checks (their tables are built with the failing flag), mixed-order
keys with honest signatures, eviction and clearing. Above the latency path's range the keyed comb
path reads a cached key's table instead of building it (any request count), so medium batches of
cached signers take 48 table additions per request instead of the Straus loop."""
import numpy as np
import pytest

from vectors import VectorGen, pack

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    from plenum_amd import _native
    _native.ensure_device()
    yield _native
    _native.KeyCache.configure(0)
    _native.set_path(_native.PV_PATH_AUTO)


def _batch(sodium, oracle, seed, n=1500):
    g = VectorGen(sodium, oracle, seed=seed)
    keys = [g.key(i) for i in range(40)]
    bad = [g.make(c)[1] for c in ("A_blacklist", "A_noncanonical", "A_offcurve", "mixed_order_A", "mixed_order_A")]
    rng = np.random.default_rng(seed)
    cases = []
    for i in range(n):
        r = rng.random()
        if r < 0.1:
            cases.append(g.make(VectorGen.CLASSES[1 + int(rng.integers(0, len(VectorGen.CLASSES) - 1))]))
        else:
            pk, sk = keys[int(rng.integers(0, len(keys)))]
            m = bytes(rng.integers(0, 256, int(rng.integers(0, 400)), dtype=np.uint8))
            sm = sodium.sign_detached(m, sk) + m
            if rng.random() < 0.05:
                sm = bytearray(sm)
                sm[int(rng.integers(0, len(sm)))] ^= 1 << int(rng.integers(0, 8))
                sm = bytes(sm)
            if rng.random() < 0.03:
                pk = bad[int(rng.integers(0, len(bad)))]
            cases.append((sm, pk))
    return cases, [k for k, _ in keys], bad


def _want(sodium, cases):
    return np.array([sodium.sign_open_ok(sm, pk) for sm, pk in cases], dtype=bool)


def test_cached_keys_bit_exact(nat, sodium, oracle):
    cases, keys, bad = _batch(sodium, oracle, seed=51)
    blob, off, pks = pack(cases)
    want = _want(sodium, cases)
    kc = nat.KeyCache
    kc.configure(128)
    kc.put(keys[:30] + bad)  # 10 signers stay uncached, the bad keys are cached with failing checks
    assert kc.stats() == (35, 128)
    assert all(kc.contains(k) for k in keys[:30]) and not kc.contains(keys[35])
    for name in ("latency", "straus", "comb", "auto"):
        nat.set_path(getattr(nat, "PV_PATH_" + name.upper()))
        got = nat.verify_sm_batch(blob, off, pks)
        assert np.array_equal(got, want), (name, np.nonzero(got != want)[0][:10])
    nat.set_path(nat.PV_PATH_AUTO)
    # cache disabled: same verdicts
    kc.enable(False)
    assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
    kc.enable(True)


def test_latency_four_wave_cached_forms(nat, sodium, oracle, monkeypatch):
    """The four-wave latency kernel (<= 512 requests, the zero-copy form Plenum's quotas and singletons
    take) on cached keys: waves 2 and 3 add the two halves of [k](-A) while wave 0 decompresses R --
    from the keys' radix-65536 rows (8 niels entries per wave) or, with the wide rows off, from the
    cached-form table (16 per wave). Single requests, a 33-request and a 300-request batch with
    cached, uncached and bad (cached, failing key checks) keys: libsodium's verdicts."""
    cases, keys, bad = _batch(sodium, oracle, seed=57)
    blob, off, pks = pack(cases)
    want = _want(sodium, cases)
    kc = nat.KeyCache
    nat.set_path(nat.PV_PATH_AUTO)
    try:
        for wide in ("1024", "0"):
            monkeypatch.setenv("PV_KC_WIDE_KEYS", wide)
            kc.configure(64)
            kc.put(keys[:30] + bad)
            for lo, hi in ((0, 1), (7, 8), (40, 73), (100, 400)):
                o = off[lo:hi + 1]
                got = nat.verify_sm_batch(blob[:int(o[-1])], o, pks[lo:hi])
                assert np.array_equal(got, want[lo:hi]), (wide, lo, hi, np.nonzero(got != want[lo:hi])[0][:10])
            for i in range(0, len(want), 37):  # one-request calls (the slot in the kernel arguments)
                o = off[i:i + 2]
                assert bool(nat.verify_sm_batch(blob[:int(o[-1])], o, pks[i:i + 1])[0]) == bool(want[i]), (wide, i)
    finally:
        monkeypatch.delenv("PV_KC_WIDE_KEYS", raising=False)
        kc.configure(0)


def test_eviction_and_clear(nat, sodium, oracle):
    cases, keys, bad = _batch(sodium, oracle, seed=52, n=800)
    blob, off, pks = pack(cases)
    want = _want(sodium, cases)
    kc = nat.KeyCache
    kc.configure(16)
    kc.put(keys)  # 40 keys into 16 slots: the last 16 put remain
    assert kc.stats() == (16, 16)
    assert all(kc.contains(k) for k in keys[-16:]) and not any(kc.contains(k) for k in keys[:24])
    kc.put(keys[:4])  # evicts the 4 least recently put
    assert all(kc.contains(k) for k in keys[:4]) and not any(kc.contains(k) for k in keys[24:28])
    nat.set_path(nat.PV_PATH_LATENCY)
    assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
    kc.clear()
    assert kc.stats() == (0, 16)
    assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
    kc.put(keys[:10] + keys[:10])  # duplicates in one call
    assert kc.stats() == (10, 16)
    assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
    nat.set_path(nat.PV_PATH_AUTO)


def _keyed_batch(sodium, oracle, seed):
    """~12k requests: 20 cached signers with ~400 requests, 10 cached with 5, 10 uncached with ~300
    (tables built in the launch), 20 uncached with 10 (Straus side), cached keys that fail
    libsodium's key checks, and ~4 % adversarial records of every class."""
    g = VectorGen(sodium, oracle, seed=seed)
    keys = [g.key(i) for i in range(60)]
    bad = [g.make(c)[1] for c in ("A_blacklist", "A_noncanonical", "A_offcurve", "mixed_order_A", "mixed_order_A")]
    rng = np.random.default_rng(seed)
    plan = [(k, 400) for k in range(20)] + [(k, 5) for k in range(20, 30)] + \
           [(k, 300) for k in range(30, 40)] + [(k, 10) for k in range(40, 60)]
    cases = []
    for k, cnt in plan:
        pk, sk = keys[k]
        for _ in range(cnt):
            m = bytes(rng.integers(0, 256, int(rng.integers(0, 320)), dtype=np.uint8))
            sm = sodium.sign_detached(m, sk) + m
            if rng.random() < 0.03:
                sm = bytearray(sm)
                sm[int(rng.integers(0, len(sm)))] ^= 1 << int(rng.integers(0, 8))
                sm = bytes(sm)
            cases.append((sm, pk))
    for j in range(150):  # honest signatures under the bad keys' bytes
        cases.append((cases[j][0], bad[j % len(bad)]))
    for _ in range(480):
        cases.append(g.make(VectorGen.CLASSES[1 + int(rng.integers(0, len(VectorGen.CLASSES) - 1))]))
    order = rng.permutation(len(cases))
    return [cases[i] for i in order], [k for k, _ in keys], bad


def test_cached_keys_on_keyed_path(nat, sodium, oracle):
    cases, keys, bad = _keyed_batch(sodium, oracle, seed=53)
    blob, off, pks = pack(cases)
    want = _want(sodium, cases)
    kc = nat.KeyCache
    kc.configure(64)
    kc.put(keys[:30] + bad)
    nat.set_path(nat.PV_PATH_AUTO)
    got = nat.verify_sm_batch(blob, off, pks)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    path, nkeys = nat.last_path()
    assert path == nat.PV_PATH_COMB
    keys_all, comb_keys, comb_req = nat.last_split()
    # every cached key (30 signers + the bad keys) plus the 10 uncached signers with ~300 requests
    assert comb_keys >= 30 + 10, (keys_all, comb_keys, comb_req)
    for name in ("comb", "straus", "latency"):
        nat.set_path(getattr(nat, "PV_PATH_" + name.upper()))
        got = nat.verify_sm_batch(blob, off, pks)
        assert np.array_equal(got, want), (name, np.nonzero(got != want)[0][:10])
    nat.set_path(nat.PV_PATH_AUTO)
    # eviction between launches: the evicted keys' requests fall back to tables built in the launch
    # or the Straus side, the newly cached ones read the cache
    kc.put(keys[30:60])  # 60 > 64 - 35 free slots: the least recently put are evicted
    assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
    kc.enable(False)
    assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
    # without the cache: a medium chunk with few distinct keys makes every key a comb key
    keys_all, comb_keys, comb_req = nat.last_split()
    assert keys_all <= 2048 and comb_keys == keys_all and comb_req == len(cases), (keys_all, comb_keys, comb_req)
    kc.enable(True)
    kc.clear()
    assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)


def test_put_failure_rolls_back(nat, sodium, oracle, monkeypatch):
    """A pv_key_cache_put that fails after building part of its keys (injected after the first
    batch's tables are scattered, over slots that evicted older keys) must leave only keys whose
    tables are built in the index: every slot the call assigned leaves the cache, the keys it did
    not touch stay, and verdicts stay libsodium's on every path; a later put succeeds normally."""
    cases, keys, bad = _batch(sodium, oracle, seed=54, n=900)
    blob, off, pks = pack(cases)
    want = _want(sodium, cases)
    kc = nat.KeyCache
    kc.configure(16)
    kc.put(keys[:16])
    monkeypatch.setenv("PV_TEST_FAIL_KC_PUT_BATCH", "0")
    with pytest.raises(nat.NativeError, match="injected failure"):
        kc.put(keys[16:24])  # evicts keys[0:8], builds keys[16:24] into their slots, then "fails"
    monkeypatch.delenv("PV_TEST_FAIL_KC_PUT_BATCH")
    assert kc.stats() == (8, 16)
    assert all(kc.contains(k) for k in keys[8:16])
    assert not any(kc.contains(k) for k in keys[:8] + keys[16:24])
    for name in ("latency", "comb", "auto"):
        nat.set_path(getattr(nat, "PV_PATH_" + name.upper()))
        got = nat.verify_sm_batch(blob, off, pks)
        assert np.array_equal(got, want), (name, np.nonzero(got != want)[0][:10])
    nat.set_path(nat.PV_PATH_AUTO)
    kc.put(keys[16:24] + bad[:3])
    assert kc.stats() == (16, 16)  # 8 free slots, then keys[8:11] evicted
    assert all(kc.contains(k) for k in keys[16:24])
    nat.set_path(nat.PV_PATH_LATENCY)
    assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
    nat.set_path(nat.PV_PATH_AUTO)
    with pytest.raises(ValueError):
        kc.contains(keys[0][:31])


def test_automatic_admission_large_host_batch(nat):
    """Automatic admission from a large host batch (a node's pipelined calls): a call above 4,096
    requests counts a sample of 4,096 of its keys, so the 1,024 signers of a 300k-request batch (~4
    sampled appearances each) are admitted behind the first call -- cached form, affine and wide rows --
    and the next calls verify from the cache (no shared per-call tables); verdicts exact throughout."""
    import nym_workload
    blob, off, pks = nym_workload.generate(0, 300000)
    bad = np.random.default_rng(9).choice(len(pks), 150, replace=False)
    blob = blob.copy()
    for i in bad:
        blob[int(off[i]) + 90] ^= 0x10
    want = np.ones(len(pks), bool)
    want[bad] = False
    kc = nat.KeyCache
    kc.configure(2048)
    kc.auto(2)
    nat.set_path(nat.PV_PATH_AUTO)
    try:
        a0, _ = kc.auto_stats()
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        a1, f1 = kc.auto_stats()
        assert a1 - a0 == 1024 and f1 == 0 and kc.stats()[0] == 1024
        for _ in range(2):
            assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        keys, comb_keys, comb_req = nat.last_split()
        assert comb_keys == keys == 1024, (keys, comb_keys, comb_req)
    finally:
        kc.auto(0)
        kc.configure(0)


def test_automatic_admission(nat, sodium, oracle, monkeypatch):
    """pv_key_cache_auto(2): a key is put into the cache behind the host batch in which it is seen
    for the second time (no manual put); verdicts are libsodium's before, during and after the
    admission (bad keys are admitted with their failing key-check flag), and a failing admission
    leaves the verdicts unchanged and the keys uncached."""
    cases, keys, bad = _batch(sodium, oracle, seed=55, n=600)
    blob, off, pks = pack(cases)
    want = _want(sodium, cases)
    kc = nat.KeyCache
    kc.configure(4096)
    kc.auto(2)
    nat.set_path(nat.PV_PATH_AUTO)
    from collections import Counter
    mult = Counter(bytes(p) for p in pks)
    distinct = set(mult)
    repeated = {k for k, c in mult.items() if c >= 2}
    assert 0 < len(repeated) < len(distinct)
    try:
        a0, _ = kc.auto_stats()
        # every appearance counts: keys seen twice within this batch are admitted behind it
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        assert kc.stats()[0] == len(repeated) and all(kc.contains(k) for k in repeated)
        assert not any(kc.contains(k) for k in distinct - repeated)
        # the next batch is verified with those tables; the keys seen once before are admitted now
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        a1, f1 = kc.auto_stats()
        assert a1 - a0 == len(distinct) and f1 == 0
        assert kc.stats()[0] == len(distinct) and all(kc.contains(k) for k in keys)
        for _ in range(2):  # now verified from the cached tables
            assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        # a failing admission: verdicts stand, nothing new is cached
        kc.clear()
        kc.auto(2)  # a new counting window
        monkeypatch.setenv("PV_TEST_FAIL_KC_PUT_BATCH", "0")
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        monkeypatch.delenv("PV_TEST_FAIL_KC_PUT_BATCH")
        a2, f2 = kc.auto_stats()
        assert a2 == a1 and f2 == len(distinct) and kc.stats()[0] == 0
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
    finally:
        kc.auto(0)
        kc.configure(0)
