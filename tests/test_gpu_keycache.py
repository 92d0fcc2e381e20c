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
    VERIFIED for the second time (no manual put); verdicts are libsodium's before, during and after
    the admission; keys that never verify (the bad keys, tampered-only appearances) are never
    admitted; a failing admission leaves the verdicts unchanged and the keys uncached."""
    cases, keys, bad = _batch(sodium, oracle, seed=55, n=600)
    blob, off, pks = pack(cases)
    want = _want(sodium, cases)
    kc = nat.KeyCache
    kc.configure(4096)
    kc.auto(2)
    nat.set_path(nat.PV_PATH_AUTO)
    from collections import Counter
    ok = Counter(bytes(pks[i]) for i in range(len(cases)) if want[i])  # verified appearances per key
    distinct = {bytes(p) for p in pks}
    verified = set(ok)
    repeated = {k for k, c in ok.items() if c >= 2}
    assert 0 < len(repeated) < len(verified) < len(distinct)
    try:
        a0, _ = kc.auto_stats()
        # keys verified twice within this batch are admitted behind it
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        assert kc.stats()[0] == len(repeated) and all(kc.contains(k) for k in repeated)
        assert not any(kc.contains(k) for k in distinct - repeated)
        # the next batch is verified with those tables; the keys verified once before are admitted now
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        a1, f1 = kc.auto_stats()
        assert a1 - a0 == len(verified) and f1 == 0
        assert kc.stats()[0] == len(verified) and all(kc.contains(k) for k in keys)
        assert not any(kc.contains(k) for k in distinct - verified)  # never verified: never admitted
        for _ in range(2):  # now verified from the cached tables
            assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        # a failing admission: verdicts stand, nothing new is cached, and the keys stay admissible
        kc.clear()
        kc.auto(2)  # a new counting window
        monkeypatch.setenv("PV_TEST_FAIL_KC_PUT_BATCH", "0")
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        monkeypatch.delenv("PV_TEST_FAIL_KC_PUT_BATCH")
        a2, f2 = kc.auto_stats()
        assert a2 == a1 and f2 >= len(verified) and kc.stats()[0] == 0
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        a3, _ = kc.auto_stats()  # the failed keys were forgotten, so they are admitted again
        assert a3 - a2 == len(verified) and kc.stats()[0] == len(verified)
    finally:
        kc.auto(0)
        kc.configure(0)


def _signed(sodium, keys, counts, seed):
    """counts[j] honest single-signature requests of ~300 bytes by keys[j] = (pk, sk)."""
    rng = np.random.default_rng(seed)
    cases = []
    for (pk, sk), c in zip(keys, counts):
        for _ in range(c):
            m = bytes(rng.integers(0, 256, 260 + int(rng.integers(0, 80)), dtype=np.uint8))
            cases.append((sodium.sign_detached(m, sk) + m, pk))
    return cases


def test_garbage_keys_admit_and_evict_nothing(nat, sodium, oracle):
    """with 1,024 signers cached (a full cache) and automatic admission on, two
    passes of 4,096 requests under 2,048 fresh garbage keys -- each key twice per pass, random
    signatures -- admit no key and evict no signer (round 5 admitted all 2,048 and evicted the
    signers: a key was counted whatever its verdict). Verdicts stay libsodium's (all rejects)."""
    g = VectorGen(sodium, oracle, seed=61)
    signers = [g.key(i) for i in range(1024)]
    kc = nat.KeyCache
    kc.configure(1024)
    nat.set_path(nat.PV_PATH_AUTO)
    try:
        kc.put([pk for pk, _ in signers])
        assert kc.stats() == (1024, 1024)
        kc.auto(2)
        rng = np.random.default_rng(62)
        garbage = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(2048)]
        a0, f0 = kc.auto_stats()
        for p in range(2):
            cases = []
            for i in range(4096):
                m = bytes(rng.integers(0, 256, 299, dtype=np.uint8))
                cases.append((bytes(rng.integers(0, 256, 64, dtype=np.uint8)) + m, garbage[(i + p) % 2048]))
            blob, off, pks = pack(cases)
            want = _want(sodium, cases)
            assert not want.any()
            assert np.array_equal(nat.verify_sm_batch(blob, off, pks), want)
        a1, f1 = kc.auto_stats()
        assert (a1 - a0, f1 - f0) == (0, 0)
        assert kc.stats() == (1024, 1024)
        assert all(kc.contains(pk) for pk, _ in signers)
        assert not any(kc.contains(k) for k in garbage)
        # the signers' own requests still verify (from the cache), tampered ones still reject
        cases = _signed(sodium, signers[:64], [4] * 64, seed=63)
        cases[5] = (cases[5][0][:70] + bytes([cases[5][0][70] ^ 1]) + cases[5][0][71:], cases[5][1])
        blob, off, pks = pack(cases)
        assert np.array_equal(nat.verify_sm_batch(blob, off, pks), _want(sodium, cases))
    finally:
        kc.auto(0)
        kc.configure(0)


def test_lru_refresh_and_readmission(nat, sodium, oracle):
    """Eviction takes the least recently USED key (launches stamp the slots they read; the stamps are
    folded into the LRU before a put evicts), and an evicted key is re-admitted on its next two
    verified appearances (round 5 kept it marked admitted until the counting window turned over)."""
    g = VectorGen(sodium, oracle, seed=64)
    keys = [g.key(i) for i in range(6)]
    kc = nat.KeyCache
    kc.configure(4)
    nat.set_path(nat.PV_PATH_AUTO)
    try:
        kc.auto(2)
        # k0..k3 admitted by their verified appearances (two each), k0 first
        for j in range(4):
            cases = _signed(sodium, [keys[j]], [2], seed=65 + j)
            blob, off, pks = pack(cases)
            assert nat.verify_sm_batch(blob, off, pks).all()
            assert kc.contains(keys[j][0])
        assert kc.stats() == (4, 4)
        # k0 is used (read from the cache), k1 is not: admitting k4 evicts k1, not k0
        for path in ("latency", "comb"):
            nat.set_path(getattr(nat, "PV_PATH_" + path.upper()))
            cases = _signed(sodium, [keys[0]], [3], seed=70)
            blob, off, pks = pack(cases)
            assert nat.verify_sm_batch(blob, off, pks).all()
        nat.set_path(nat.PV_PATH_AUTO)
        cases = _signed(sodium, [keys[4]], [2], seed=71)
        blob, off, pks = pack(cases)
        assert nat.verify_sm_batch(blob, off, pks).all()
        assert kc.contains(keys[4][0]) and kc.contains(keys[0][0])
        assert not kc.contains(keys[1][0])
        # k1 comes back: re-admitted on its next two verified appearances
        cases = _signed(sodium, [keys[1]], [1], seed=72)
        blob, off, pks = pack(cases)
        assert nat.verify_sm_batch(blob, off, pks).all()
        assert not kc.contains(keys[1][0])
        assert nat.verify_sm_batch(blob, off, pks).all()
        assert kc.contains(keys[1][0])
        # a tampered appearance does not count
        cases = _signed(sodium, [keys[5]], [3], seed=73)
        cases = [(c[0][:80] + bytes([c[0][80] ^ 4]) + c[0][81:], c[1]) for c in cases]
        blob, off, pks = pack(cases)
        assert not nat.verify_sm_batch(blob, off, pks).any()
        assert not kc.contains(keys[5][0])
    finally:
        kc.auto(0)
        kc.configure(0)
