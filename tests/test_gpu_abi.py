"""GPU tests of the C ABI's ordering and multi-GPU contracts, and of the keyed path's slot mapping
at its boundaries (include/plenum_verify.h):
  * pv_memcpy_d2h right after pv_verify_batch_device, with no pv_sync, returns the launch's verdicts
    (library stream and a caller stream);
  * pv_memcpy_h2d right after a launch does not change the inputs that launch reads;
  * pv_verify_batch_multi_gpu on a one-device mask (the box has one GPU) is bit-exact against
    libsodium 1.0.18 on the configs[2] batch, and ReqAuthenticator.authenticate_batch(devices=[0])
    returns the reference's golden outcomes;
  * keyed-comb slot ranges that straddle 256-slot tiles and 2,048-slot XCD rounds at every offset
    mod 2,048, and a dedup workgroup whose LDS key table overflows (the direct-atomic fallback)."""
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
    _native.set_path(_native.PV_PATH_AUTO)
    return _native


@pytest.fixture(scope="module")
def nym256k():
    import nym_workload
    return nym_workload.generate(0, 1 << 18)


def _tampered(blob, off, idx, byte=70):
    b = blob.copy()
    for i in idx:
        b[int(off[i]) + byte] ^= 0x04
    return b


def test_copy_back_ordered_without_sync(native, nym256k):
    """pv_verify_batch_device enqueues on the library's non-blocking stream (or a caller stream);
    pv_memcpy_d2h issued straight after it must wait for the launch, not read stale words."""
    from bench import DeviceBatch, bits
    blob, off, pks = nym256k
    n = len(off) - 1
    bad = np.random.default_rng(2).choice(n, 300, replace=False)
    want = np.ones(n, bool)
    want[bad] = False
    db = DeviceBatch(_tampered(blob, off, bad), off, pks)
    L = native.lib()
    import ctypes
    s = ctypes.c_void_p()
    native.check(L.pv_stream_create(ctypes.byref(s)), "pv_stream_create")
    try:
        stale = np.full(db.words, 0xA5A5A5A5A5A5A5A5, np.uint64)
        for stream in (None, s):
            native.check(L.pv_memcpy_h2d(db.d_verdict, stale.ctypes.data, stale.nbytes), "h2d")
            native.check(L.pv_verify_batch_device(db.d_blob, db.d_off, n, db.d_pk, db.d_verdict, stream),
                         "pv_verify_batch_device")
            got = bits(db.verdict_words(), n)  # no pv_sync / pv_stream_sync
            assert np.array_equal(got, want), (stream, np.nonzero(got != want)[0][:10])
    finally:
        native.check(L.pv_stream_destroy(s), "pv_stream_destroy")
        db.free()


def test_upload_after_launch_keeps_inputs(native, nym256k):
    """Overwriting a batch's device inputs with pv_memcpy_h2d right after its launch: the launch
    still verifies the first batch (all valid but 300 tampered), the next launch the second (all
    tampered)."""
    from bench import DeviceBatch, bits
    blob, off, pks = nym256k
    n = len(off) - 1
    bad = np.random.default_rng(3).choice(n, 300, replace=False)
    first = _tampered(blob, off, bad)
    second = _tampered(blob, off, range(n), byte=71)
    want = np.ones(n, bool)
    want[bad] = False
    db = DeviceBatch(first, off, pks)
    L = native.lib()
    try:
        db.verify()
        native.check(L.pv_memcpy_h2d(db.d_blob, second.ctypes.data, second.nbytes), "h2d")
        assert np.array_equal(bits(db.verdict_words(), n), want)
        db.verify()
        assert not bits(db.verdict_words(), n).any()
    finally:
        db.free()


def test_multi_gpu_one_device_config3_bit_exact(native, oracle):
    """pv_verify_batch_multi_gpu with the one GPU of this box (its context is the primary's; one
    shard, the ncclCommInitAll clique of one device, the in-place all-gather and the copy-back from
    the first device) on configs[2]: 1M requests with 2 % adversarial records, every verdict equal
    to libsodium's."""
    import nym_workload
    from adversarial import inject
    from oracle.oracle import cpu_verdicts
    blob, off, pks = nym_workload.generate(0, 1 << 20)
    blob2, pks2, idx, _ = inject(blob, off, pks, 0.02, seed=3, oracle=oracle)
    want = cpu_verdicts(blob2, off, pks2)
    assert native.ensure_devices([0]) == (0,)
    n_dev = native.lib().pv_multi_gpu_devices(None, 0)
    assert n_dev == 1
    assert native.multi_gpu_clique() == {"devices": [0], "nranks": 1, "user_ranks": [0]}  # RCCL's own count
    got = native.verify_sm_batch_multi(blob2, off, pks2)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    # odd sizes: a partial last verdict word, fewer requests than one word
    for k in (1, 63, 65, 4097, 100001):
        o = off[:k + 1]
        got = native.verify_sm_batch_multi(blob2[:int(o[-1])], o, pks2[:k])
        assert np.array_equal(got, want[:k]), k
    # the single-device calls still work on the shared context afterwards
    assert np.array_equal(native.verify_sm_batch(blob2[:int(off[3000])], off[:3001], pks2[:3000]), want[:3000])


def test_authenticate_batch_on_device_list(native):
    """ReqAuthenticator.authenticate_batch(items, devices=[0]) (the multi-GPU engine) returns the
    reference's golden outcomes, exceptions included."""
    from plenum_amd.client_authn import CoreAuthNr
    from plenum_amd.req_authenticator import ReqAuthenticator
    from plenum_amd.state_utils import DictState
    with open(os.path.join(HERE, "golden", "reqauth.json")) as f:
        ra_data = json.load(f)
    for seq in ra_data["seqs"]:
        ra = ReqAuthenticator()
        # (the golden's NoAuthenticatorFound sequence has no authenticator registered)
        if seq["items"] and len(seq["out"]) > 1 or seq["out"][0].get("exc") != "NoAuthenticatorFound":
            core = CoreAuthNr(["1", "101"], ["105"], ["action"], state=DictState({}))
            for idr, vk in ra_data["clients"].items():
                core.addIdr(idr, vk)
            ra.register_authenticator(core)
        res = ra.authenticate_batch([(json.loads(json.dumps(r)), k) for r, k in seq["items"]], devices=[0])
        got = [({"exc": type(x).__name__, "msg": str(x)} if isinstance(x, Exception) else {"set": sorted(x)})
               for x in res]
        assert got == seq["out"]


def _keyed_records(sodium, n_keys, per_key, seed, bad_every=13, shuffle=True):
    """n_keys fresh keys with per_key requests each (records alternate between the key's valid
    signature and a tampered copy by position), shuffled (else key-minor: keys 0..n_keys-1, then
    again, ...). Returns blob, off, pks, expected."""
    rng = np.random.default_rng(seed)
    good, badr, keys = [], [], []
    for k in range(n_keys):
        pk, sk = sodium.seed_keypair(rng.bytes(32))
        m = rng.bytes(int(rng.integers(0, 400)))
        sm = sodium.sign_detached(m, sk) + m
        t = bytearray(sm)
        t[int(rng.integers(0, len(t)))] ^= 1 << int(rng.integers(0, 8))
        good.append(sm)
        badr.append(bytes(t))
        keys.append(pk)
    want_good = np.array([sodium.sign_open_ok(good[k], keys[k]) for k in range(n_keys)])
    want_bad = np.array([sodium.sign_open_ok(badr[k], keys[k]) for k in range(n_keys)])
    assert want_good.all() and not want_bad.any()
    kk = np.tile(np.arange(n_keys), per_key)
    jj = np.repeat(np.arange(per_key), n_keys)
    tam = (jj * 7 + kk) % bad_every == 0
    if shuffle:
        perm = rng.permutation(len(kk))
        kk, tam = kk[perm], tam[perm]
    recs = [badr[k] if t else good[k] for k, t in zip(kk, tam)]
    lens = np.fromiter((len(r) for r in recs), np.uint64, len(recs))
    off = np.zeros(len(recs) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    blob = np.frombuffer(b"".join(recs), np.uint8)
    pks = np.frombuffer(b"".join(keys), np.uint8).reshape(n_keys, 32)[kk]
    return blob, off, np.ascontiguousarray(pks), ~tam


def test_comb_slot_ranges_at_every_tile_and_xcd_offset(native, sodium):
    """Every key has 257 requests, so in the key-sorted slot order the keys' slot ranges start at
    257 j: with 2,048 keys they start at EVERY offset mod 2,048 (257 is odd), i.e. every position
    within a 256-slot tile and within a round of 8 tiles over the 8 XCDs (the mapping the dropped
    work-queue variant of comb_a got wrong with a period of 2,048 requests). Positions inside each key
    alternate valid / tampered records, so a request verified with another slot's digits or point
    gets the wrong verdict. AUTO (every key a comb key) and forced COMB, bit-exact. Device-resident
    inputs (pv_verify_batch_device): the whole batch is ONE launch chunk (a host-buffer call of this
    size is cut into pipelined sub-batches)."""
    from bench import DeviceBatch, bits
    blob, off, pks, want = _keyed_records(sodium, 2048, 257, seed=77)
    n = len(off) - 1
    assert n == 2048 * 257
    db = DeviceBatch(blob, off, pks)
    try:
        for path in (native.PV_PATH_AUTO, native.PV_PATH_COMB):
            native.set_path(path)
            db.verify()
            got = bits(db.verdict_words(), n)
            split = native.last_split()
            native.set_path(native.PV_PATH_AUTO)
            assert np.array_equal(got, want), (path, np.nonzero(got != want)[0][:10])
            assert split == (2048, 2048, n), (path, split)
    finally:
        db.free()
    # the same batch from host buffers (pipelined sub-batches: each a keyed chunk of its own)
    assert np.array_equal(native.verify_sm_batch(blob, off, pks), want)


def test_dedup_lds_table_overflow(native, sodium):
    """4,096 distinct keys in each 4,096-request workgroup of the LDS-aggregated dedup insert: its
    4,096-entry LDS table fills up and the requests whose 64 probes fail take their rank with a
    direct device atomic (the mixed LDS-base / direct rank path). Forced COMB (every key a comb
    key), bit-exact; keys' two requests fall in different workgroups."""
    blob, off, pks, want = _keyed_records(sodium, 4096, 2, seed=78, bad_every=3, shuffle=False)
    n = len(off) - 1
    native.set_path(native.PV_PATH_COMB)
    try:
        got = native.verify_sm_batch(blob, off, pks)
        split = native.last_split()
    finally:
        native.set_path(native.PV_PATH_AUTO)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert split == (4096, 4096, n), split
