"""GPU: the node-side key cache (pv_key_cache_*). A cached key is verified on the latency path with
32 comb-table additions instead of 252 doublings; verdicts must stay exactly libsodium's, including
keys that fail libsodium's key checks (their tables are built with the failing flag), mixed-order
keys with honest signatures, eviction and clearing. The throughput paths never read the cache."""
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
