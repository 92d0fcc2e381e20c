"""GPU parity: the HIP engine's verdicts vs libsodium 1.0.18 (the reference's own native verifier,
nacl_wrappers.py:108) and the C oracle, on seeded normal + adversarial vectors. Calls go through
the C ABI (libplenum_verify.so) via plenum_amd._native."""
import numpy as np
import pytest

from vectors import VectorGen, pack

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["straus", "comb", "latency"])
def native(request):
    """The engine with each arithmetic path forced in turn (verdicts must not depend on it)."""
    from plenum_amd import _native
    _native.ensure_device()
    _native.set_path(getattr(_native, "PV_PATH_" + request.param.upper()))
    yield _native
    _native.set_path(_native.PV_PATH_AUTO)


def reference_verdicts(sodium, cases):
    return np.array([sodium.sign_open_ok(sm, pk) for sm, pk in cases], dtype=bool)


def test_each_adversarial_class(native, sodium, oracle):
    g = VectorGen(sodium, oracle, seed=11)
    cases = []
    for cls in VectorGen.CLASSES:
        cases += [g.make(cls) for _ in range(24)]
    blob, off, pks = pack(cases)
    got = native.verify_sm_batch(blob, off, pks)
    want = reference_verdicts(sodium, cases)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(VectorGen.CLASSES[i // 24], cases[i][0].hex(), cases[i][1].hex(), want[i]) for i in bad[:5]]
    # the classes that must be rejected are, and mixed-order keys pass ~1/8 of the time
    assert want.sum() > 24 * 3


def test_each_adversarial_class_small_batches(native, sodium, oracle):
    """Per class, a batch of 16 (at or below PV_LAT4_MAX: the latency path's four-wave form, where
    [k1](+-A) and [k2](-R') are each cut at 2^68; the other paths run their usual kernels), mixed-order
    A and R with passing and failing signatures included."""
    g = VectorGen(sodium, oracle, seed=12)
    for cls in VectorGen.CLASSES:
        cases = [g.make(cls) for _ in range(16)]
        blob, off, pks = pack(cases)
        got = native.verify_sm_batch(blob, off, pks)
        want = reference_verdicts(sodium, cases)
        assert np.array_equal(got, want), (cls, np.nonzero(got != want)[0][:5])


def test_four_wave_cutoff_sizes(native, sodium, oracle):
    """Batches on both sides of the latency path's four-wave / two-wave cutoff (PV_LAT4_MAX = 512,
    and the round-3 cutoff 256), 2 % adversarial records included."""
    g = VectorGen(sodium, oracle, seed=19)
    cases = g.batch(513, adversarial_frac=0.02)
    want = reference_verdicts(sodium, cases)
    for n in (256, 257, 511, 512, 513):
        blob, off, pks = pack(cases[:n])
        got = native.verify_sm_batch(blob, off, pks)
        assert np.array_equal(got, want[:n]), (n, np.nonzero(got != want[:n])[0][:10])


def test_mixed_batch_2pct(native, sodium, oracle):
    g = VectorGen(sodium, oracle, seed=12)
    cases = g.batch(3000, adversarial_frac=0.02)
    blob, off, pks = pack(cases)
    got = native.verify_sm_batch(blob, off, pks)
    want = reference_verdicts(sodium, cases)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


def test_unaligned_offsets_and_ragged(native, sodium, oracle):
    g = VectorGen(sodium, oracle, seed=13)
    cases = [g.valid(g.msg(0, 300)) for _ in range(200)] + [g.make("short_sm") for _ in range(20)]
    g.rng.shuffle(cases)
    # leading garbage so that record starts are at every residue mod 8
    blob, off, pks = pack(cases)
    blob2 = np.concatenate([np.full(3, 0xAA, np.uint8), blob])
    got = native.verify_sm_batch(blob2, off + 3, pks)
    want = reference_verdicts(sodium, cases)
    assert np.array_equal(got, want)


def test_empty_and_single(native, sodium, oracle):
    g = VectorGen(sodium, oracle, seed=14)
    assert native.verify_sm_batch(np.zeros(0, np.uint8), np.zeros(1, np.uint64), np.zeros((0, 32), np.uint8)).size == 0
    for n in (1, 63, 64, 65, 257):
        cases = g.batch(n, adversarial_frac=0.3)
        blob, off, pks = pack(cases)
        assert np.array_equal(native.verify_sm_batch(blob, off, pks), reference_verdicts(sodium, cases))


def test_repeated_keys_with_adversarial(native, sodium, oracle):
    """Few distinct keys shared by many requests (the comb path's case), including shared keys that
    fail libsodium's key checks, honest signatures under mixed-order keys, and per-request
    signature corruption, at every record alignment."""
    g = VectorGen(sodium, oracle, seed=15)
    base = [g.make("valid") for _ in range(40)]
    bad_keys = [g.make(c)[1] for c in ("A_blacklist", "A_noncanonical", "A_offcurve", "mixed_order_A")]
    cases = []
    rng = np.random.default_rng(15)
    for i in range(4000):
        sm, pk = base[int(rng.integers(0, len(base)))]
        r = rng.random()
        if r < 0.04:
            pk = bad_keys[int(rng.integers(0, len(bad_keys)))]
        elif r < 0.08:
            sm = bytearray(sm)
            sm[int(rng.integers(0, len(sm)))] ^= 1 << int(rng.integers(0, 8))
            sm = bytes(sm)
        cases.append((sm, pk))
    blob, off, pks = pack(cases)
    got = native.verify_sm_batch(blob, off, pks)
    want = reference_verdicts(sodium, cases)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert 0.85 * len(cases) < want.sum() < len(cases)


def _long_record_cases(sodium, oracle, lengths, seed):
    g = VectorGen(sodium, oracle, seed=seed)
    cases = []
    for ln in lengths:
        sm, pk = g.valid(bytes(g.rng.getrandbits(8) for _ in range(ln)))
        cases.append((sm, pk))
        bad = bytearray(sm)
        bad[-1 if ln else 0] ^= 0x10
        cases.append((bytes(bad), pk))
    return cases


def test_small_calls_zero_copy_records(native, sodium, oracle):
    """Small host-buffer calls whose records all fit a zero-copy slot (sm <= 1,840 bytes: the slot's
    2,048-byte stride holds the 48-byte header, the record and the hash's 160-byte read-ahead, which
    ends exactly at the slot's edge for the longest records): on the latency path the call IS
    zero-copy (the kernel reads the pinned slots over PCIe and copies each record into LDS), valid
    and tampered records, every alignment. pv_last_zero_copy says which form ran."""
    lengths = list(range(1700, 1777, 4)) + [1776, 0, 1, 127, 128]
    cases = _long_record_cases(sodium, oracle, lengths, seed=16)
    assert max(len(sm) for sm, _ in cases) == 1840
    blob, off, pks = pack(cases)
    want = reference_verdicts(sodium, cases)
    assert want.sum() == len(cases) // 2
    for lead in (0, 1, 2, 3):
        blob2 = np.concatenate([np.full(lead, 0x55, np.uint8), blob])
        got = native.verify_sm_batch(blob2, off + lead, pks)
        assert np.array_equal(got, want), (lead, np.nonzero(got != want)[0][:8])
        assert native.last_zero_copy() == (native.last_path()[0] == native.PV_PATH_LATENCY), lead


def test_one_request_calls(native, sodium, oracle):
    """One-request host-buffer calls (verifySignature singletons): a slot of <= 1,024 bytes (records
    up to 816 bytes) travels in the kernel arguments (pv_lat4_one_kernel), longer ones in a pinned
    slot; valid and tampered records on both sides of that edge, every alignment, each call alone."""
    lengths = [0, 1, 127, 128, 300, 700, 744, 748, 752, 756, 760, 800]
    cases = _long_record_cases(sodium, oracle, lengths, seed=18)
    want = reference_verdicts(sodium, cases)
    assert want.sum() == len(cases) // 2
    assert any(len(sm) <= 816 for sm, _ in cases) and any(len(sm) > 816 for sm, _ in cases)
    for i, (sm, pk) in enumerate(cases):
        blob, off, pks = pack([(sm, pk)])
        for lead in (0, 1, 2, 3):
            blob2 = np.concatenate([np.full(lead, 0x55, np.uint8), blob])
            got = native.verify_sm_batch(blob2, off + lead, pks)
            assert bool(got[0]) == bool(want[i]), (len(sm), lead)
            assert native.last_zero_copy() == (native.last_path()[0] == native.PV_PATH_LATENCY), (len(sm), lead)


def test_small_calls_long_records(native, sodium, oracle):
    """Small host-buffer calls with records beyond a zero-copy slot (1,841 bytes up to 9 KB): the
    whole call takes the staged copy form (the zero-copy choice is made per call from the longest
    record), valid and tampered, at every alignment."""
    lengths = list(range(1780, 1960, 20)) + [4000, 9000]
    cases = _long_record_cases(sodium, oracle, lengths, seed=17)
    blob, off, pks = pack(cases)
    want = reference_verdicts(sodium, cases)
    assert want.sum() == len(cases) // 2
    for lead in (0, 1, 2, 3):
        blob2 = np.concatenate([np.full(lead, 0x55, np.uint8), blob])
        got = native.verify_sm_batch(blob2, off + lead, pks)
        assert np.array_equal(got, want), (lead, np.nonzero(got != want)[0][:8])
        assert not native.last_zero_copy()


def test_encode_wave_edges(native, sodium, oracle):
    """Batch sizes at the encode kernel's wave edges (8 points per lane, 512 requests per wave, the wave's
    64 lane products inverted together: PvWaveInvert), with lanes and whole groups past the batch's end and
    rejected records (whose points are left out of the products) on both sides of each edge."""
    g = VectorGen(sodium, oracle, seed=20)
    cases = g.batch(2113, adversarial_frac=0.1)
    want = reference_verdicts(sodium, cases)
    for n in (448, 449, 1023, 1024, 1025, 1537, 2048, 2113):
        blob, off, pks = pack(cases[:n])
        got = native.verify_sm_batch(blob, off, pks)
        assert np.array_equal(got, want[:n]), (n, np.nonzero(got != want[:n])[0][:10])
