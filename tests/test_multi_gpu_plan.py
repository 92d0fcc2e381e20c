"""CPU tests of the single-process multi-GPU entry (pv_init_devices / pv_verify_batch_multi_gpu,
include/plenum_verify.h): its shard plan is the multi-process harness's (plenum_amd/sharding.py)
for 2 and 8 devices and every batch size class, the gathered words reassemble into the global
bitmap, and without a GPU the entry and the authenticate_batch(devices=...) surface fail loudly."""
import numpy as np
import pytest

from plenum_amd import _native
from plenum_amd.sharding import assemble, shard_bounds, words_per_rank


@pytest.mark.parametrize("ndev", [1, 2, 8])
def test_shard_plan_matches_sharding(ndev):
    for n in (0, 1, 63, 64, 65, 127, 513, 4095, 4097, 100001, 1 << 20, (1 << 26) + 17):
        bounds, wpr = _native.shard_plan(n, ndev)
        assert len(bounds) == ndev + 1 and bounds[0] == 0 and bounds[-1] == n
        assert [int(b) for b in bounds[:-1]] == [shard_bounds(n, ndev, r)[0] for r in range(ndev)]
        assert wpr == words_per_rank(n, ndev)
        for r in range(ndev):
            lo, hi = int(bounds[r]), int(bounds[r + 1])
            assert lo % 64 == 0 and hi >= lo  # whole verdict words: shard r's bits start at word lo / 64
            assert (hi - lo + 63) // 64 <= wpr


@pytest.mark.parametrize("ndev", [2, 8])
def test_gathered_words_reassemble(ndev):
    """What pv_verify_batch_multi_gpu does after its all-gather (shard r at r * wpr words, the bytes
    of shard r copied to bit bounds[r]) gives the same bitmap as the multi-process assemble()."""
    rng = np.random.default_rng(ndev)
    for n in (1, 64, 1000, 70001):
        verdicts = rng.random(n) < 0.7
        bounds, wpr = _native.shard_plan(n, ndev)
        gathered = np.zeros((ndev, wpr), np.uint64)
        for r in range(ndev):
            lo, hi = int(bounds[r]), int(bounds[r + 1])
            bits = np.zeros(wpr * 64, np.uint8)
            bits[:hi - lo] = verdicts[lo:hi]
            gathered[r] = np.packbits(bits, bitorder="little").view(np.uint64)
        out = np.zeros((n + 7) // 8, np.uint8)
        raw = gathered.view(np.uint8).reshape(ndev, -1)
        for r in range(ndev):
            lo, hi = int(bounds[r]), int(bounds[r + 1])
            if hi > lo:
                out[lo // 8:lo // 8 + (hi - lo + 7) // 8] = raw[r, :(hi - lo + 7) // 8]
        got = np.unpackbits(out, bitorder="little")[:n].astype(bool)
        assert np.array_equal(got, verdicts)
        assert np.array_equal(assemble(gathered, n, ndev), verdicts)


def test_shard_plan_rejects_bad_device_counts():
    with pytest.raises(_native.NativeError):
        _native.shard_plan(100, 0)
    with pytest.raises(_native.NativeError):
        _native.shard_plan(100, 17)


def test_multi_gpu_entry_without_gpu_fails_loudly():
    L = _native.lib()
    if L.pv_device_count() > 0:
        pytest.skip("a GPU is visible")
    assert L.pv_init_devices(0x3) < 0
    assert L.pv_multi_gpu_devices(None, 0) == 0
    blob = np.zeros(64, np.uint8)
    off = np.array([0, 64], np.uint64)
    with pytest.raises(_native.NativeUnavailable):
        _native.verify_sm_batch_multi(blob, off, np.zeros((1, 32), np.uint8), devices=[0, 1])
    from plenum_amd.client_authn import CoreAuthNr
    from plenum_amd.req_authenticator import ReqAuthenticator
    core = CoreAuthNr(["1"], ["105"], [], state=None)
    core.addIdr("4QxzWk3ajdnEA37NdNU5Kt", "~BqfrxmXgj5A1hq4KpmaxWK")
    ra = ReqAuthenticator()
    ra.register_authenticator(core)
    req = {"identifier": "4QxzWk3ajdnEA37NdNU5Kt", "reqId": 1, "operation": {"type": "1"},
           "signature": "3" * 87, "protocolVersion": 2}
    with pytest.raises(_native.NativeUnavailable):
        ra.authenticate_batch([(req, "k")], devices=[0, 1])
