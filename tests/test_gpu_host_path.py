"""GPU tests of the host-fed path (include/plenum_verify.h pv_verify_batch, pv_host_alloc /
pv_host_register, pv_verify_batch_multi_gpu) and of its failure paths:
  * large host batches are verified in pipelined sub-batches (H2D of sub-batch j on the copy stream
    beside the kernels of j - 1); every input form -- pageable numpy, all inputs in the library's
    pinned arena, an arena sub-range whose offsets do not start at 0, only the blob pinned, a numpy
    buffer registered in place -- gives libsodium 1.0.18's verdicts on a configs[2]-style batch
    (2 % adversarial records), at sizes that leave a ragged last sub-batch and a partial verdict word;
  * an injected staging failure (pv_test_inject) after the first sub-batch is in flight returns an
    error, and the next call -- single-device and the multi-GPU entry -- is bit-exact;
  * pv_init_devices with a device that does not exist fails without touching the primary context;
  * released arena blocks are handed out again by size (the pinned block cache) and verify bit-exact;
  * with >= 2 GPUs (skipped on a one-GPU box): the multi-GPU entry with empty shards, a partial last
    word and a >= 8 MB blob is bit-exact."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from plenum_amd import _native
    _native.ensure_device()
    _native.set_path(_native.PV_PATH_AUTO)
    return _native


@pytest.fixture(scope="module")
def adv400k(oracle):
    """400,000 NYM requests (~145 MB of records: three pipelined sub-batches), 2 % adversarial, and
    libsodium's verdicts."""
    import nym_workload
    from adversarial import inject
    from oracle.oracle import cpu_verdicts
    blob, off, pks = nym_workload.generate(0, 400000)
    blob2, pks2, _, _ = inject(blob, off, pks, 0.02, seed=5, oracle=oracle)
    return blob2, off, pks2, cpu_verdicts(blob2, off, pks2)


def _check(got, want, what):
    assert np.array_equal(got, want), (what, np.nonzero(got != want)[0][:10])


def test_host_forms_bit_exact(native, adv400k):
    blob, off, pks, want = adv400k
    A = native.HostArena
    # pageable
    _check(native.verify_sm_batch(blob, off, pks), want, "pageable")
    # the whole batch in the arena (offsets from 0: DMA'd as they are)
    ab, ao, ak = A.batch(blob, off, pks)
    assert A.is_pinned(ab) and A.is_pinned(ao) and A.is_pinned(ak)
    assert not A.is_pinned(blob)
    _check(native.verify_sm_batch(ab, ao, ak), want, "arena")
    # a sub-range of the arena batch whose offsets start past 0 (rebased in staging), ragged sizes
    for lo, hi in ((131072 + 64, 400000), (1, 262144 + 1 + 77), (64 * 5000 + 3, 64 * 5000 + 3 + 140000)):
        _check(native.verify_sm_batch(ab, ao[lo:hi + 1], ak[lo:hi]), want[lo:hi], ("arena range", lo, hi))
    # only the blob pinned (keys and offsets pageable)
    _check(native.verify_sm_batch(ab, np.array(ao), np.array(ak)), want, "blob pinned")
    # a numpy buffer pinned in place
    reg = np.array(blob)
    L = native.lib()
    native.check(L.pv_host_register(reg.ctypes.data, reg.nbytes), "pv_host_register")
    try:
        assert A.is_pinned(reg)
        _check(native.verify_sm_batch(reg, off, pks), want, "registered")
    finally:
        native.check(L.pv_host_unregister(reg.ctypes.data), "pv_host_unregister")
    assert not A.is_pinned(reg)
    assert L.pv_host_free(ctypes.c_void_p(reg.ctypes.data)) != 0  # not an arena block


def test_arena_blocks_reused_after_free(native, adv400k):
    """pv_host_free keeps a released block pinned for the next pv_host_alloc of a similar size (at
    most twice the request); a released block is no longer reported as the caller's pinned memory;
    a batch built in reused blocks is verified bit-exact."""
    import gc
    blob, off, pks, want = adv400k
    L = native.lib()

    def alloc(nbytes):
        p = ctypes.c_void_p()
        native.check(L.pv_host_alloc(ctypes.byref(p), nbytes), "pv_host_alloc")
        return p.value

    a = alloc(48 << 20)
    native.check(L.pv_host_free(ctypes.c_void_p(a)), "pv_host_free")
    assert L.pv_host_is_pinned(ctypes.c_void_p(a), 1) == 0
    b = alloc(40 << 20)
    assert b == a and L.pv_host_is_pinned(ctypes.c_void_p(a), 48 << 20) == 1
    c = alloc(8 << 20)  # 48 MB > 2 x 8 MB: a new block
    assert c != a
    for q in (b, c):
        native.check(L.pv_host_free(ctypes.c_void_p(q)), "pv_host_free")
    n = 300000
    o = off[:n + 1]
    first = native.HostArena.batch(blob[:int(o[-1])], o, pks[:n])
    addrs = sorted(x.ctypes.data for x in first)
    del first
    gc.collect()
    ab, ao, ak = native.HostArena.batch(blob[:int(o[-1])], o, pks[:n])
    assert sorted(x.ctypes.data for x in (ab, ao, ak)) == addrs
    _check(native.verify_sm_batch(ab, ao, ak), want[:n], "reused arena")


def test_injected_stage_failure_then_exact(native, adv400k, monkeypatch):
    monkeypatch.setenv("PV_ENABLE_TEST_HOOKS", "1")
    blob, off, pks, want = adv400k
    k = 262144 + 999
    o = off[:k + 1]
    for n in (k, 3000, 20000):  # pipelined, quota-size (one DMA), medium (one piece)
        on = off[:n + 1]
        native.inject_stage_failures(0, 1)
        with pytest.raises(native.NativeError, match="injected"):
            native.verify_sm_batch(blob[:int(on[-1])], on, pks[:n])
        _check(native.verify_sm_batch(blob[:int(on[-1])], on, pks[:n]), want[:n], ("after failure", n))
    # the multi-GPU entry: one shard's staging fails, the call errors, the next one is exact
    devs = native.ensure_devices([0])
    native.inject_stage_failures(devs[0], 1)
    with pytest.raises(native.NativeError, match="injected"):
        native.verify_sm_batch_multi(blob[:int(o[-1])], o, pks[:k])
    _check(native.verify_sm_batch_multi(blob[:int(o[-1])], o, pks[:k]), want[:k], "multi after failure")
    _check(native.verify_sm_batch(blob[:int(o[-1])], o, pks[:k]), want[:k], "single after multi failure")
    native.inject_stage_failures(0, 0)


def test_init_devices_bad_mask_keeps_primary(native, adv400k):
    blob, off, pks, want = adv400k
    L = native.lib()
    ndev = L.pv_device_count()
    for mask in (1 << ndev, (1 << ndev) | 1, 0, 1 << 20):
        assert L.pv_init_devices(mask) < 0, mask
    # the primary context and the multi-GPU clique built before are unaffected
    o = off[:5001]
    _check(native.verify_sm_batch(blob[:int(o[-1])], o, pks[:5000]), want[:5000], "primary after bad mask")
    assert native.ensure_devices([0]) == (0,)
    _check(native.verify_sm_batch_multi(blob[:int(o[-1])], o, pks[:5000]), want[:5000], "multi after bad mask")


def test_pipelined_shared_tables_with_one_off_keys(native, sodium):
    """A pipelined host call whose first sub-batch has more than 2,048 distinct keys (1,024 signers
    with ~100 requests each plus ~25k one-off keys): the first sub-batch gives tables only to the
    signers (>= 48 requests) and publishes them; the later sub-batches read the signers' tables from
    the shared store and verify their one-off keys on the Straus path in the same launches -- forced
    COMB too (every key a comb key up to the capacity) -- libsodium's verdicts."""
    from test_gpu_configs import _split_batch
    from oracle.oracle import cpu_verdicts
    blob, off, pks = _split_batch(sodium, 262144, 60000, seed=17)
    want = cpu_verdicts(blob, off, pks)
    assert 0 < (~want).sum() < len(want) // 50
    for path in (native.PV_PATH_AUTO, native.PV_PATH_COMB):
        native.set_path(path)
        try:
            got = native.verify_sm_batch(blob, off, pks)
        finally:
            native.set_path(native.PV_PATH_AUTO)
        _check(got, want, ("one-off keys", path))


def test_pipelined_partly_warm_cache(native, adv400k):
    """a pipelined host call with half of its signers in the node-side key cache. The later
    sub-batches look a key up in the node cache first and in the call's shared store next
    (pv_key_cache_probe_kernel's two views), so the uncached signers' tables are built once per call, not
    once per sub-batch (round 5 turned sharing off whenever the cache held a key). Verdicts are
    libsodium's on AUTO and forced COMB; the call is no slower than with the cache empty."""
    import time
    blob, off, pks, want = adv400k
    keys, counts = np.unique(pks, axis=0, return_counts=True)
    signers = [bytes(k) for k, c in zip(keys, counts) if c >= 100]
    assert len(signers) >= 1000
    kc = native.KeyCache

    def timed_calls():
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            got = native.verify_sm_batch(blob, off, pks)
            ts.append(time.perf_counter() - t0)
            _check(got, want, "partly warm")
        return float(np.median(ts))

    try:
        kc.configure(2048)
        native.verify_sm_batch(blob, off, pks)  # warm: staging sized
        cold = timed_calls()
        kc.put(signers[::2])
        assert kc.stats()[0] == len(signers[::2])
        for path in (native.PV_PATH_AUTO, native.PV_PATH_COMB):
            native.set_path(path)
            try:
                _check(native.verify_sm_batch(blob, off, pks), want, ("partly warm", path))
            finally:
                native.set_path(native.PV_PATH_AUTO)
        warm = timed_calls()
        print("pipelined 400k call: cache empty %.2f ms, half the signers cached %.2f ms" % (1e3 * cold, 1e3 * warm))
        assert warm < 1.25 * cold, (warm, cold)
    finally:
        kc.configure(0)


def test_multi_gpu_two_or_more_devices(native, adv400k):
    L = native.lib()
    G = L.pv_device_count()
    if G < 2:
        pytest.skip("one GPU visible: the multi-device clique needs >= 2")
    blob, off, pks, want = adv400k
    devs = native.ensure_devices(range(G))
    assert native.multi_gpu_clique() == {"devices": list(devs), "nranks": G, "user_ranks": list(range(G))}
    for n in (1, 63, 64 * G - 1, 64 * G + 65, 100001, len(want)):  # empty shards, partial words, >= 8 MB
        o = off[:n + 1]
        _check(native.verify_sm_batch_multi(blob[:int(o[-1])], o, pks[:n], devs), want[:n], ("multi", n))
