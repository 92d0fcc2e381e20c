"""bench.py — Ed25519 request verifies/sec on MI355X (BASELINE.json metric), one process per GPU.

A step = one pass of the hot path over one batch: pv_verify_batch_device on this rank's shard of
device-resident synthetic NYM-style signed requests, and for N > 1 the one RCCL all-gather of the
per-shard verdict bitmaps. N = 1 runs configs[1] of BASELINE.json (1M requests);
N > 1 runs configs[4] (64M requests split into N contiguous 64-aligned shards, i.e. 8M per GPU at
N = 8: fixed total work). About 0.1 % of the records are tampered so the verdict check compares
bitmaps, not "all ones". Inputs are uploaded to HBM before the timed region; host serialization and
PCIe are reported separately, never as `value`. Beside the headline at N = 1: configs[2] (2 %
adversarial, verdicts compared with libsodium's), configs[3] (3 signatures per request), the
forced Straus path, host-buffer latency and the CPU baselines. The multi-GPU harness uses no
framework: rank 0's RCCL id travels through a file, barriers and the max over ranks are RCCL
all-gathers (class Comm).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--per-gpu REQUESTS]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]

import bench_constants as BC  # noqa: E402
import nym_workload  # noqa: E402
from plenum_amd import _native  # noqa: E402

METRIC = "Ed25519 request verifies/sec (1/2/4/8 MI355X) + % int-VALU peak"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class DeviceBatch:
    """Device-resident copy of one shard (library-owned allocations, no framework tensors)."""

    def __init__(self, blob, off, pks):
        L = _native.lib()
        self.n = len(off) - 1
        self.ptrs = []
        self.d_blob = self._put(blob, blob.nbytes + _native.PV_BLOB_SLACK)
        self.d_off = self._put(off, off.nbytes)
        self.d_pk = self._put(pks, pks.nbytes)
        self.words = (self.n + 63) // 64
        self.d_verdict = self._alloc(self.words * 8)
        self.L = L

    def _alloc(self, nbytes):
        p = ctypes.c_void_p()
        _native.check(_native.lib().pv_dev_alloc(ctypes.byref(p), nbytes), "pv_dev_alloc")
        self.ptrs.append(p)
        return p

    def _put(self, arr, nbytes):
        p = self._alloc(nbytes)
        arr = np.ascontiguousarray(arr)
        _native.check(_native.lib().pv_memcpy_h2d(p, arr.ctypes.data, arr.nbytes), "pv_memcpy_h2d")
        return p

    def verify(self):
        _native.check(self.L.pv_verify_batch_device(self.d_blob, self.d_off, self.n, self.d_pk, self.d_verdict, None),
                      "pv_verify_batch_device")

    def verdict_words(self, ptr=None, words=None):
        words = words or self.words
        out = np.zeros(words, dtype=np.uint64)
        _native.check(self.L.pv_memcpy_d2h(out.ctypes.data, ptr or self.d_verdict, out.nbytes), "pv_memcpy_d2h")
        return out

    def free(self):
        for p in self.ptrs:
            self.L.pv_dev_free(p)


def usable_cpus():
    """(affinity, quota, usable): the CPUs in this process's affinity set, the cgroup CPU quota in CPUs
    (cgroup v2 cpu.max or v1 cfs_quota_us / cfs_period_us; None = unlimited or unreadable), and the
    number of threads that can actually run at once = min of the two. A GPU box shares its host with
    other tenants: its affinity set can show the whole machine (256 CPUs) while the cgroup grants ~16,
    and libsodium on 256 threads then runs SLOWER than on 16 (profiles/r06/mid/bench.json: 0.30 M/s on 256 threads against 0.50 M/s on 16)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except Exception:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except Exception:
            pass
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return aff, quota, usable


def cpu_baseline(blob, off, pks, sample, target_s=10.0, config3=None, share=16, share_s=5.0):
    """libsodium 1.0.18 crypto_sign_open (the reference's verifier) over the first `sample` requests of
    the same workload, repeated until about `target_s` seconds have run, on every host CPU this process
    can use (the host's nproc = the affinity set, capped by the cgroup CPU quota when the
    box grants fewer CPUs than it shows: usable_cpus) -- `value` and `cores`; when the affinity set is
    larger than that, also on the whole affinity set (`all_affinity_threads`, oversubscribed); then on
    `share` threads (the per-GPU share of the node's cores, 128 / 8 on the MI355X nodes) for about
    `share_s` seconds -- `per_gpu_share`. The C oracle on one thread if libsodium is absent.
    With config3 = (blob, off, pks), also libsodium's per-record verdicts over that whole batch (one
    pass on every CPU, timed and returned): the reference outputs the config-3 leg's GPU verdicts are
    checked against."""
    from oracle.libsodium_ref import LibSodium, find_libsodium
    from oracle.oracle import Oracle, cpu_verdicts
    o = Oracle()
    fn = o.lib.cpu_baseline_run
    fn.restype = ctypes.c_int64
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_uint64, ctypes.c_int]
    path = find_libsodium()
    aff, quota, nproc = usable_cpus()
    use_sodium = path is not None
    if not use_sodium:
        sample = min(sample, 2000)
        aff = nproc = share = 1
    off_s = np.ascontiguousarray(off[:sample + 1])

    def run(threads, seconds):
        passes, acc, dt = 0, 0, 0.0
        while dt < seconds and passes < 1000:  # repeat passes until ~seconds of CPU work has run
            t0 = time.perf_counter()
            acc += fn((path or "").encode(), 1 if use_sodium else 0, blob.ctypes.data, off_s.ctypes.data,
                      pks.ctypes.data, sample, threads)
            dt += time.perf_counter() - t0
            passes += 1
        return passes, acc, dt

    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        pass
    version = LibSodium(path).version if use_sodium else None
    impl = "libsodium %s at %s" % (version, path) if use_sodium else "C oracle restatement"
    # the thread count that gets the most out of this host: one short pass at 16, 32, 64, ... threads up
    # to the usable count (a box can show more CPUs than it grants without a readable quota)
    sweep = {}
    if use_sodium and nproc > 16:
        t = 16
        while True:
            m = min(sample, 8192 * t)
            t0 = time.perf_counter()
            fn(path.encode(), 1, blob.ctypes.data, off_s.ctypes.data, pks.ctypes.data, m, t)
            sweep[t] = round(m / (time.perf_counter() - t0), 1)
            if t >= nproc:
                break
            t = min(2 * t, nproc)
        best = max(sweep, key=sweep.get)
        if best != nproc:
            nproc = best
    passes, acc, dt = run(nproc, target_s)
    out = {"value": round(sample * passes / dt, 1), "unit": "verifies/s", "cores": nproc,
           "kind": "reference" if use_sodium else "port",
           "sample": "%d passes over %d requests of the same synthetic NYM workload, crypto_sign_open on %d "
                     "threads (%s: affinity set %d, cgroup quota %s) (%s), %s" % (
                         passes, sample, nproc,
                         "the best of a 16, 32, 64, ... thread sweep up to every CPU this process can use" if sweep
                         else "every CPU this process can use",
                         aff, "none" if quota is None else "%.1f CPUs" % quota, cpu_model, impl),
           "cpu_model": cpu_model, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
           "thread_sweep_verifies_per_s": {str(k): v for k, v in sweep.items()},
           "accepted": int(acc), "seconds": round(dt, 3)}
    if aff != nproc:
        ap_, aa, adt = run(aff, share_s)
        out["all_affinity_threads"] = {"value": round(sample * ap_ / adt, 1), "cores": aff, "accepted": int(aa),
                                       "seconds": round(adt, 3),
                                       "note": "the same loop on every CPU of the affinity set: more threads than "
                                               "the cgroup quota lets run at once"}
    share = min(share, nproc)
    if share != nproc:
        sp, sa, sdt = run(share, share_s)
        out["per_gpu_share"] = {"value": round(sample * sp / sdt, 1), "cores": share, "accepted": int(sa),
                                "seconds": round(sdt, 3),
                                "note": "the same libsodium loop on %d threads: one GPU's share of an 8-GPU node's "
                                        "128 cores" % share}
    verdicts = None
    if config3 is not None:
        t0 = time.perf_counter()
        verdicts = cpu_verdicts(*config3, threads=nproc)
        c3 = time.perf_counter() - t0
        out["config3"] = {"requests": len(verdicts), "verifies_per_s": round(len(verdicts) / c3, 1),
                          "accepted": int(verdicts.sum()), "seconds": round(c3, 3),
                          "note": "one pass of crypto_sign_open over the whole configs[2] batch on %d threads; "
                                  "these verdicts are what the GPU's config3 verdicts are compared with" % nproc}
    return out, verdicts


def ingress_leg(n, blob, off, wire, steps, warmup):
    """what happens before pv_verify_batch_device, measured on the same workload.
      host   C++ signing serialization + Request.digest of every received JSON request
             (pv_signing_serialize_json, 16 threads) — the host-serialization overhead
      device pv_ingress_verify_device: GPU base58 decode of every signature, key resolution for
             the 1,024 signers, sm assembly, verification (inputs resident in HBM)
      e2e    authenticate_wire_packed (JSON bytes -> identifier sets, Python glue included) on the
             whole batch; authenticate_wire_batch (dicts decoded) and one_call_per_request on 64k
    Returns the bench-line object."""
    from plenum_amd.client_authn import CoreAuthNr
    from plenum_amd.req_authenticator import ReqAuthenticator
    from plenum_amd.wire import (PV_SER_REQUEST, authenticate_wire_batch, authenticate_wire_packed,
                                 signing_serialize_packed)
    L = _native.lib()
    wblob, woff, sblob, soff = wire
    threads = min(16, len(os.sched_getaffinity(0)))
    signing_serialize_packed(wblob[:int(woff[1024])], woff[:1025], PV_SER_REQUEST, threads)
    t0 = time.perf_counter()
    st, mblob, moff, _ = signing_serialize_packed(wblob, woff, PV_SER_REQUEST, threads)
    ser_s = time.perf_counter() - t0
    # the serializer's messages must be the ones the requests were signed over
    starts = off[:-1] + 64
    same = bool((st == 0).all()) and np.array_equal(np.diff(moff), off[1:] - starts)
    if same:
        idx = np.arange(0, n, 4099)
        same = all(mblob[int(moff[i]):int(moff[i + 1])].tobytes() == blob[int(starts[i]):int(off[i + 1])].tobytes()
                   for i in idx)
    pool = nym_workload._pool()
    idrs = [p["did"].encode() for p in pool]
    vks = [p["abbr"].encode() for p in pool]
    ib, io = _native._blob(idrs)
    vb, vo = _native._blob(vks)
    vp = np.ones(len(pool), np.uint8)
    msg_idx = np.arange(n, dtype=np.uint32)
    signer_idx = (np.arange(n, dtype=np.uint64) % len(pool)).astype(np.uint32)
    db = DeviceBatch(np.zeros(1, np.uint8), np.zeros(2, np.uint64), np.zeros((1, 32), np.uint8))
    d = {k: db._put(a, a.nbytes) for k, a in (("s", sblob), ("so", soff), ("m", mblob[:int(moff[-1]) + 8]),
                                                ("mo", moff), ("mi", msg_idx), ("si", signer_idx), ("i", ib),
                                                ("io", io), ("v", vb), ("vo", vo), ("vp", vp))}
    d_status = db._alloc(n)
    d_ver = db._alloc((n + 63) // 64 * 8)
    mtotal = int(moff[-1])

    def step():
        _native.check(L.pv_ingress_verify_device(d["s"], d["so"], d["mi"], d["si"], n, d["m"], d["mo"], n, mtotal,
                                                 d["i"], d["io"], d["v"], d["vo"], d["vp"], len(pool), d_status,
                                                 d_ver, None), "pv_ingress_verify_device")

    for _ in range(warmup):
        step()
    _native.check(L.pv_sync(), "pv_sync")
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _native.check(L.pv_sync(), "pv_sync")
    dev_s = (time.perf_counter() - t0) / steps
    front = ctypes.c_double()
    _native.check(L.pv_ingress_front_ms(ctypes.byref(front)), "pv_ingress_front_ms")
    status = np.zeros(n, np.uint8)
    _native.check(L.pv_memcpy_d2h(status.ctypes.data, d_status, n), "pv_memcpy_d2h")
    ver = np.unpackbits(db.verdict_words(d_ver, (n + 63) // 64).view(np.uint8), bitorder="little")[:n]
    db.free()
    # end to end through the Python surface: the whole batch from wire bytes (authenticate_wire_packed),
    # then a 64k sample through the list API (every dict decoded) and in the reference's
    # one-authenticate-call-per-request mode

    def make_ra():
        core = CoreAuthNr(["1"], ["105"], [], state=None)
        for p in pool:
            core.addIdr(p["did"], p["abbr"])
        ra = ReqAuthenticator()
        ra.register_authenticator(core)
        return ra

    def expected_ids(results, lo=0):
        return all(r == {pool[(lo + i) % len(pool)]["did"]} for i, r in enumerate(results))

    authenticate_wire_packed(make_ra(), wblob, woff, threads)  # warm-up: device buffers sized, pages touched
    tm = {}
    t0 = time.perf_counter()
    packed = authenticate_wire_packed(make_ra(), wblob, woff, threads, timings=tm)
    e2e_s = time.perf_counter() - t0
    e2e_ok = expected_ids(packed.results)
    del packed
    k = min(n, 1 << 16)
    raws = [wblob[int(woff[i]):int(woff[i + 1])].tobytes() for i in range(k)]
    lists = {}
    for mode, once in (("list_api", False), ("one_call_per_request", True)):
        t0 = time.perf_counter()
        res = authenticate_wire_batch(make_ra(), raws, threads=threads, one_call_per_request=once)
        dt = time.perf_counter() - t0
        lists[mode] = {"requests": k, "requests_per_s": round(k / dt, 1),
                       "ok": bool(expected_ids([r for _, r in res]))}
    return {
        "host_signing_serialize": {"requests": n, "threads": threads, "seconds": round(ser_s, 4),
                                   "requests_per_s": round(n / ser_s, 1),
                                   "us_per_request_per_thread": round(ser_s * threads * 1e6 / n, 3),
                                   "messages_match_signed": bool(same)},
        "device_ingress": {"verifies_per_s": round(n / dev_s, 1), "ms_per_step": round(dev_s * 1e3, 3),
                           "front_end_ms": round(front.value, 4),
                           "note": "GPU b58 decode + key resolution + sm assembly + verification, HBM-resident",
                           "verdicts_ok": bool((status == 0).all() and ver.all())},
        "wire_batch_e2e": {"requests": n, "requests_per_s": round(n / e2e_s, 1), "threads": threads,
                           "stages_s": {x: round(tm[x], 4) for x in ("serialize_s", "plan_s", "gpu_s", "finish_s")},
                           "ok": bool(e2e_ok),
                           "note": "authenticate_wire_packed: wire bytes -> identifier sets and the verified-request "
                                   "cache; C++ plan on `threads` threads, one GPU launch, Python per distinct "
                                   "signer/type and per request only for the result objects (request dicts of "
                                   "device-finished requests decoded on access)"},
        "wire_batch_list_api": dict(lists["list_api"], note="authenticate_wire_batch: every request dict decoded "
                                                            "(json.loads) in the call"),
        "wire_batch_one_call_per_request": dict(lists["one_call_per_request"],
                                                note="the reference's call pattern: ReqAuthenticator.authenticate "
                                                     "once per request, signature checks batched in one launch"),
    }


H2D_PEAK_BPS = 57.5e9  # one pinned hipMemcpyAsync of 400 MB on the MI355X box (profiles/r05/h2d_bw.txt)


def host_path_leg(blob, off, pks, want, reps=7):
    """SURVEY.md §8e host traffic at N = 1: the whole configs[1] batch from host buffers through
    pv_verify_batch (H2D of 262,144-request sub-batches, the first and last half-size, on a copy
    stream beside the previous sub-batch's kernels, verdicts back), median of `reps` calls per form
    after one that sizes the staging, the two forms alternating call by call (the box's PCIe is
    shared with other tenants' GPUs: a slow stretch hits both forms alike):
      arena     the batch built in the library's pinned arena (pv_host_alloc: what a node that
                receives into such buffers gets; the DMA reads the caller's bytes, no staging copy)
      pageable  the same bytes in ordinary numpy memory (copy workers stage each sub-batch first)
    Never `value`: the headline is device-resident."""
    n = len(off) - 1
    h2d_bytes = int(off[-1] - off[0]) + 32 * n + 8 * (n + 1)
    t0 = time.perf_counter()
    ab, ao, ak = _native.HostArena.batch(blob, off, pks)
    fill_s = time.perf_counter() - t0
    forms = {"pageable": (blob, off, pks), "arena": (ab, ao, ak)}
    ts = {f: [] for f in forms}
    ok = {f: True for f in forms}
    for f, (b, o, k) in forms.items():
        _native.verify_sm_batch(b, o, k)
    for _ in range(reps):
        for f, (b, o, k) in forms.items():
            t1 = time.perf_counter()
            v = _native.verify_sm_batch(b, o, k)
            ts[f].append(time.perf_counter() - t1)
            ok[f] &= bool(np.array_equal(v, want))
    del forms, ab, ao, ak

    def stats(f):
        med = float(np.median(ts[f]))
        return {"verifies_per_s": round(n / med, 1), "median_ms": round(1e3 * med, 3),
                "min_ms": round(1e3 * min(ts[f]), 3), "effective_h2d_GBps": round(h2d_bytes / med / 1e9, 2),
                "ok": ok[f]}
    arena, page = stats("arena"), stats("pageable")
    return dict(arena, requests=n, ok=arena["ok"] and page["ok"], form="arena", h2d_bytes=h2d_bytes,
                pcie_bound_verifies_per_s=round(n / (h2d_bytes / H2D_PEAK_BPS), 1),
                frac_of_pcie_bound=round(arena["verifies_per_s"] / (n / (h2d_bytes / H2D_PEAK_BPS)), 4),
                arena_fill_s=round(fill_s, 3), pageable=page,
                note="pv_verify_batch on the headline batch (tampered records included, verdicts checked) from "
                     "host memory, PCIe included; pipelined sub-batches of 262,144 requests (first and last "
                     "half-size), arena and pageable calls alternating; pcie_bound = the H2D bytes at the "
                     "box's measured %.1f GB/s" % (H2D_PEAK_BPS / 1e9))


def multisig_reduce(bits_nk):
    """authenticate_multi with threshold None (client_authn.py:84-118) over verdict bits (n, k) in
    dict order: a request is accepted iff all k signatures verify; a rejected one raises
    InsufficientCorrectSignatures(k, #correct, {incorrect signers}). Returns (accepted bool[n],
    correct count int[n])."""
    return bits_nk.all(axis=1), bits_nk.sum(axis=1)


def multisig_leg(multi, n_req, k, steps):
    """configs[3]: n_req requests with k signatures each (authenticate_multi, threshold None = all),
    expanded to one record per (request, signer) and verified in one pv_verify_batch_device call
    per step; ~1 % of the records carry a corrupted signature (seeded positions among the k), so the
    check compares the device's record bitmap with the known bits and the per-request reduction
    (accepted iff all k verify; #correct of a rejected request) with the expected one. Reported
    beside the headline, never as `value`."""
    blob, off, pks, bad = multi
    mb = DeviceBatch(blob, off, pks)
    mb.verify()  # warm-up
    _native.check(_native.lib().pv_sync(), "pv_sync")
    t0 = time.perf_counter()
    for _ in range(steps):
        mb.verify()
    _native.check(_native.lib().pv_sync(), "pv_sync")
    dt = (time.perf_counter() - t0) / steps
    path, nkeys = _native.last_path()
    got = bits(mb.verdict_words(), n_req * k).reshape(n_req, k)
    mb.free()
    acc, correct = multisig_reduce(got)
    want_acc, want_correct = multisig_reduce(~bad)
    records_ok = bool(np.array_equal(got, ~bad))
    reduce_ok = bool(np.array_equal(acc, want_acc) and np.array_equal(correct, want_correct))
    return {"requests": n_req, "signatures_per_request": k, "verifies_per_s": round(n_req * k / dt, 1),
            "requests_per_s": round(n_req / dt, 1), "ms_per_step": round(dt * 1e3, 3), "steps": steps,
            "distinct_keys": nkeys, "corrupted_records": int(bad.sum()),
            "requests_accepted": int(acc.sum()), "requests_rejected": int((~acc).sum()),
            "expected_rejected": int((~want_acc).sum()),
            "record_bitmap_ok": records_ok, "reduction_ok": reduce_ok, "verdicts_ok": records_ok and reduce_ok,
            "note": "configs[3]: 1 author + 2 endorsers over the same payload, records request-major, "
                    "device-resident, one launch per step; ~1 % of records have a flipped R/S bit"}


def config1_python(wire, k=10000, gpu=False):
    """configs[0] of BASELINE.json: k signed NYM requests through CoreAuthNr.authenticate one at a
    time on one host core, each signature checked by libsodium 1.0.18 crypto_sign_open (what the
    reference's node does per request: json.loads -> Request -> ReqAuthenticator.authenticate ->
    DidVerifier -> libnacl). The drop-in Python classes stand in for the reference's (golden-pinned
    in tests/test_host_logic.py); libsodium is called through ctypes as libnacl does. CPU leg only.
    gpu=True: the same loop with the HIP engine and no batch context -- the unmodified drop-in per-call
    pattern (nacl_wrappers.py:232-242 inside client_authn.py:84-118, reached from node.py:2624): every
    signature is one pv_verify_batch call of ONE request (the zero-copy latency kernel)."""
    from oracle.libsodium_ref import LibSodium, find_libsodium
    from plenum_amd import batch
    from plenum_amd.client_authn import CoreAuthNr
    from plenum_amd.req_authenticator import ReqAuthenticator
    from plenum_amd.wire import Request
    if find_libsodium() is None and not gpu:
        return None
    sodium = None if gpu else LibSodium()
    wblob, woff = wire[0], wire[1]
    k = min(k, len(woff) - 1)
    pool = nym_workload._pool()
    core = CoreAuthNr(["1"], ["105"], [], state=None)
    for p in pool:
        core.addIdr(p["did"], p["abbr"])
    ra = ReqAuthenticator()
    ra.register_authenticator(core)
    raws = [wblob[int(woff[i]):int(woff[i + 1])].tobytes() for i in range(k)]

    def engine(blob, off, pks):  # one crypto_sign_open per call, as libnacl.crypto_sign_open
        return [sodium.sign_open_ok(blob.tobytes(), pks[0].tobytes())]

    ok = 0
    if gpu:  # no batch context: plenum_amd.batch.verdict() makes one engine call per signature
        for raw in raws[:200]:  # warm-up: staging sized, clocks up
            req = Request(**json.loads(raw.decode()))
            ra.authenticate(req.as_dict, req.key)
        ra = ReqAuthenticator()
        ra.register_authenticator(core)
        t0 = time.perf_counter()
        for i, raw in enumerate(raws):
            req = Request(**json.loads(raw.decode()))
            ok += ra.authenticate(req.as_dict, req.key) == {pool[i % len(pool)]["did"]}
        dt = time.perf_counter() - t0
        return {"requests": k, "cores": 1, "requests_per_s": round(k / dt, 1),
                "us_per_request": round(dt * 1e6 / k, 1), "accepted": ok,
                "note": "configs[0] through the drop-in surface with the HIP engine and NO batching: per-request "
                        "json.loads + Request + ReqAuthenticator.authenticate, each signature one pv_verify_batch "
                        "call of one request (what an unmodified Node.verifySignature gets; the feed points "
                        "authenticate_client_quota / authenticate_propagates batch instead)"}
    t0 = time.perf_counter()
    with batch.active(batch.VerdictCache(), engine):
        for i, raw in enumerate(raws):
            req = Request(**json.loads(raw.decode()))
            ok += ra.authenticate(req.as_dict, req.key) == {pool[i % len(pool)]["did"]}
    dt = time.perf_counter() - t0
    return {"requests": k, "cores": 1, "requests_per_s": round(k / dt, 1), "us_per_request": round(dt * 1e6 / k, 1),
            "accepted": ok, "note": "configs[0]: per-request json.loads + Request + ReqAuthenticator.authenticate "
                                    "(drop-in classes) + libsodium crypto_sign_open, one host thread"}


_C1_WIRE = None


def _config1_worker(_):
    return config1_python(_C1_WIRE)


def config1_legs(wire, share=16):
    """configs[0] on one core, then on one forked process per CPU this process can use (usable_cpus:
    SURVEY §8d(i)'s nproc, capped by the cgroup quota) and on `share` processes (one GPU's share of the node's cores);
    each process runs the same 10k requests with its own authenticators, aggregate = all requests /
    wall time. Runs before the GPU comes up."""
    import multiprocessing as mp
    global _C1_WIRE
    one = config1_python(wire)
    if one is None:
        return None
    _, _, nproc = usable_cpus()

    def pool(procs):
        t0 = time.perf_counter()
        with mp.get_context("fork").Pool(procs) as p:
            parts = p.map(_config1_worker, range(procs))
        dt = time.perf_counter() - t0
        total = sum(x["requests"] for x in parts)
        return {"processes": procs, "requests": total, "requests_per_s": round(total / dt, 1),
                "accepted": sum(x["accepted"] for x in parts),
                "note": "wall time incl. process start; each process authenticates the same 10k requests"}

    _C1_WIRE = wire
    try:
        one["processes"] = pool(max(1, nproc))
        if min(share, nproc) != nproc:
            one["processes_per_gpu_share"] = pool(max(1, min(share, nproc)))
    finally:
        _C1_WIRE = None
    return one


def _pmc_kernel(kernels, name):
    """The PMC summary entry of kernel `name` (template instances are keyed "void name<W>")."""
    if name in kernels:
        return kernels[name]
    for k, v in kernels.items():
        if k.startswith("void %s<" % name):
            return v
    return {}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary, if present:
    2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: on gfx950 FETCH_SIZE counts half the bytes of
    16-B/lane streaming reads, the access width of every table and message load here)."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        k = _pmc_kernel(d.get("kernels", {}), kernel)
        return k.get("hbm_bytes_per_launch_corrected", k.get("hbm_bytes_per_launch"))
    except Exception:
        return None


def pmc_valu_issue(kernel, cus=256):
    """VALU issue rate of `kernel` from the committed PMC summary: wave-instructions (SQ_INSTS_VALU) per
    CU-cycle over its dispatch under the counters (eff. clock = GRBM_GUI_ACTIVE / dispatch time). The
    ceiling depends on the instruction mix: measured ~2.6 cycles per wave64 VOP2 and
    ~4.9 per VOP3-class instruction (v_mad_u64_u32, v_mul_lo_u32, v_lshrrev_b64) per SIMD, i.e. ~1.5
    VOP2 or ~0.8 VOP3 instructions per CU-cycle over 4 SIMDs (profiles/r01_isa_rates_full.jsonl): a
    value near the mix's ceiling means the kernel is bound by instruction issue, not memory."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            k = _pmc_kernel(json.load(f)["kernels"], kernel)
        c = k["counters_per_dispatch"]
        return round(c["SQ_INSTS_VALU"] / (k["median_dispatch_s_under_pmc"] * k["eff_clock_GHz"] * 1e9 * cus), 3)
    except Exception:
        return None


FUSED_MIN_REQ = 262144  # pv_comb_ab_kernel runs for chunks above this (PV_FUSED_MIN_REQ), else pv_comb_a_kernel
CONFIG5_TOTAL = 1 << 26  # configs[4]: 64M requests over the node's GPUs


class Comm:
    """Multi-GPU harness without a framework: the RCCL communicator of libplenum_verify is the only
    channel. Rank 0's ncclUniqueId reaches the other ranks through a file named after the job
    (PV_BENCH_JOB from bench.py's own launcher, else the launcher's PID and port:
    torch.distributed.run starts every rank of one job from the same agent process, so the name is
    unique per job and never stale); barrier = a one-word all-gather + device sync; the max over
    ranks of a host time = an all-gather of every rank's time."""

    def __init__(self, world, rank, L):
        import tempfile
        self.world, self.rank, self.L = world, rank, L
        job = os.environ.get("PV_BENCH_JOB") or "%d_%s" % (os.getppid(), os.environ.get("MASTER_PORT", "0"))
        path = os.path.join(tempfile.gettempdir(), "pv_bench_%s.uid" % job)
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            _native.check(L.pv_comm_unique_id(uid), "pv_comm_unique_id")
            with open(path + ".tmp", "wb") as f:
                f.write(bytes(uid))
            os.replace(path + ".tmp", path)
        else:
            t0 = time.time()
            while not os.path.exists(path):
                if time.time() - t0 > 300:
                    raise TimeoutError("rank %d: no communicator id from rank 0 at %s" % (rank, path))
                time.sleep(0.05)
            with open(path, "rb") as f:
                uid = (ctypes.c_uint8 * 128).from_buffer_copy(f.read())
        _native.check(L.pv_comm_init(world, rank, uid), "pv_comm_init")
        self.path = path
        self.d_one, self.d_all = ctypes.c_void_p(), ctypes.c_void_p()
        _native.check(L.pv_dev_alloc(ctypes.byref(self.d_one), 8), "pv_dev_alloc")
        _native.check(L.pv_dev_alloc(ctypes.byref(self.d_all), 8 * world), "pv_dev_alloc")

    def allgather_u64(self, v):
        x = np.array([v], np.uint64)
        _native.check(self.L.pv_memcpy_h2d(self.d_one, x.ctypes.data, 8), "pv_memcpy_h2d")
        _native.check(self.L.pv_allgather_verdicts(self.d_one, 1, self.d_all, None), "pv_allgather_verdicts")
        _native.check(self.L.pv_sync(), "pv_sync")
        out = np.zeros(self.world, np.uint64)
        _native.check(self.L.pv_memcpy_d2h(out.ctypes.data, self.d_all, 8 * self.world), "pv_memcpy_d2h")
        return out

    def rccl_ranks(self):
        """Every rank's (ncclCommCount, ncclCommUserRank) of its communicator, gathered."""
        nr, rk = _native.comm_count()
        both = self.allgather_u64((nr << 32) | rk)
        return [int(x) >> 32 for x in both], [int(x) & 0xFFFFFFFF for x in both]

    def barrier(self):
        self.allgather_u64(self.rank)

    def max_f64(self, x):
        return float(self.allgather_u64(np.float64(x).view(np.uint64)).view(np.float64).max())

    def close(self):
        self.barrier()
        self.L.pv_dev_free(self.d_one)
        self.L.pv_dev_free(self.d_all)
        self.L.pv_comm_destroy()
        if self.rank == 0 and os.path.exists(self.path):
            os.remove(self.path)


def hbm_in_use():
    """(bytes in use, total) on this process's current HIP device (hipMemGetInfo from the HIP runtime the
    engine already loaded; device-wide, so other processes' allocations on the GPU count too), or None."""
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        free, total = ctypes.c_size_t(), ctypes.c_size_t()
        if hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) != 0:
            return None
        return total.value - free.value, total.value
    except OSError:
        return None


def rccl_summary(world, nranks_by_rank, user_rank_by_rank):
    """The N > 1 line's `rccl` object: what RCCL itself reported on every rank (ncclCommCount /
    ncclCommUserRank through pv_comm_count), so the line shows the all-gather ran over `world` ranks."""
    return {"nranks": nranks_by_rank[0], "rank": user_rank_by_rank[0],
            "nranks_max_over_ranks": max(nranks_by_rank), "nranks_min_over_ranks": min(nranks_by_rank),
            "user_ranks": list(user_rank_by_rank),
            "ok": bool(min(nranks_by_rank) == max(nranks_by_rank) == world and
                       sorted(user_rank_by_rank) == list(range(world)))}


def tamper_count(n):
    return max(1, n // 1024)


def expected_bits(n, rank):
    """The headline batch's verdicts by construction: every request valid except the
    tamper_count(n) records adversarial_batch.tamper() corrupted (seed 1000 + rank)."""
    idx = np.random.default_rng(1000 + rank).choice(n, size=min(tamper_count(n), n), replace=False)
    want = np.ones(n, bool)
    want[idx] = False
    return want


def bits(words, n):
    return np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)


def config3_leg(db_like, blob0, off, pks, steps, warmup, timed_fn):
    """configs[2]: the headline's 1M requests with 2 % adversarial records (tools/adversarial_batch.py,
    every SURVEY §8c(iv) class, mixed-order keys forged with libsodium), verified in the default AUTO
    mode. Timed like the headline; verdicts returned for the check against libsodium (cpu_baseline)."""
    import adversarial_batch
    t0 = time.perf_counter()
    blob3, pks3, idx, labels = adversarial_batch.inject(blob0, off, pks, 0.02, seed=3)
    prep_s = time.perf_counter() - t0
    db3 = DeviceBatch(blob3, off, pks3)
    n = len(off) - 1
    _native.set_path(_native.PV_PATH_AUTO)
    # the same warmup and step count as the headline: the first passes over a freshly allocated
    # batch run ~10 % slower (a 1+5-step leg read 3.17 ms/step, 5+20 steps 2.85-2.90 ms;
    # profiles/r03/half/ab_config3_side)
    for _ in range(max(1, warmup)):
        db3.verify()
    el, _ = timed_fn(steps, db3.verify, stages=False)
    _, st = timed_fn(steps, db3.verify)
    keys, comb_keys, comb_req = _native.last_split()
    got = bits(db3.verdict_words(), n)
    db3.free()
    res = {"value": round(n * steps / el, 1), "unit": "verifies/s", "steps": steps,
           "ms_per_step": round(1e3 * el / steps, 3), "requests": n, "adversarial": int(len(idx)),
           "classes": sorted(set(labels)), "accepted": int(got.sum()),
           "split": {"distinct_keys": keys, "comb_keys": comb_keys, "comb_requests": comb_req,
                     "straus_requests": n - comb_req},
           "stages_ms": {s: round(v, 4) for s, v in st.items()}, "batch_prep_s": round(prep_s, 2)}
    return res, got, (blob3, off, pks3)


def workload_name(n, world):
    return ("configs[1]: %d single-sig NYM-style requests (~299 B signing-serialized, 1024 signer DIDs)" % n
            if world == 1 else
            "configs[4]: %d single-sig NYM-style requests sharded over %d GPUs (%d per GPU, contiguous "
            "64-aligned shards), verdict bitmaps all-gathered with RCCL every step" % (n * world, world, n))


def assemble_result(world, n, steps, warmup, elapsed, stage_ms, chunks, comb, nkeys, record_bytes_avg,
                    ok_local, ok_all, per_gpu_fixed=False, fused=False):
    """The headline bench line from the measured quantities (every rank count; the optional legs are
    added by the caller): value = requests of all ranks / the max-over-ranks time of `steps` steps,
    the roofline of the dominant kernel from its HIP-event launch time (stage "msm" / chunks), the
    whole-pipeline figures from the stage times. fused: the comb path's MSM stage is pv_comb_ab_kernel
    ([S]B and [k](-A) in one kernel), else pv_comb_a_kernel ([k](-A) only)."""
    total = n * world * steps
    value = total / elapsed
    ms_per_step = 1e3 * elapsed / steps
    mac_kernel = ((BC.MAC_COMB_AB_KERNEL if fused else BC.MAC_COMB_MSM_KERNEL) if comb
                  else BC.MAC_MSM_HALF_KERNEL)
    launch_ms = stage_ms["msm"] / chunks  # the roofline kernel's average launch (one per chunk)
    achieved = mac_kernel * (n / chunks) / (launch_ms * 1e-3)
    pipeline_ms = sum(stage_ms.values())
    per_gpu_rate = n / (pipeline_ms * 1e-3)
    mac_executed = (BC.MAC_COMB_MSM + BC.MAC_ENCODE / 4 + BC.MAC_COMB_PER_KEY * nkeys / (n / chunks)) if comb \
        else (BC.MAC_PER_VERIFY - BC.MAC_ENCODE * 3 / 4)
    kernel = ("pv_comb_ab_kernel" if fused else "pv_comb_a_kernel") if comb else "pv_msm_kernel"
    return {
        "metric": METRIC, "value": round(value, 1), "unit": "verifies/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak" if world == 1 or per_gpu_fixed else "strong",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": workload_name(n, world) + ", %d of them tampered (must-reject), device-resident" % (
                       tamper_count(n) * world),
                   "requests_per_gpu": n, "global_batch": n * world, "parallelism": "dp%d" % world,
                   "chunks_per_gpu_step": chunks, "record_bytes_avg": round(record_bytes_avg, 1),
                   "path": "keyed comb (%d distinct keys per chunk, tables built inside every step)" % nkeys if comb
                   else "per-request Straus"},
        "roofline": {"bound": "valu", "kernel": kernel,
                     "achieved": round(achieved / 1e12, 3), "peak": round(BC.PEAK_MAC_PER_S / 1e12, 3),
                     "unit": "TMAC/s (v_mad_u64_u32 int32 MACs)", "frac": round(achieved / BC.PEAK_MAC_PER_S, 4),
                     "traffic": pmc_traffic(kernel),
                     "algorithmic_mac_per_verify": round(mac_kernel), "launch_ms": round(launch_ms, 4),
                     "frac_of_measured_mad_stream": round(achieved / BC.MEASURED_MAD_STREAM_MAC_PER_S, 4),
                     "valu_issue_per_cu_cycle_pmc": pmc_valu_issue(kernel)},
        "pipeline": {**{s + "_ms": round(v, 4) for s, v in stage_ms.items()},
                     "kernel_verifies_per_s_per_gpu": round(per_gpu_rate, 1),
                     "whole_pipeline_valu_frac": round(mac_executed * per_gpu_rate / BC.PEAK_MAC_PER_S, 4),
                     "libsodium_equivalent_mac_rate_over_peak": round(
                         BC.MAC_PER_VERIFY * per_gpu_rate / BC.PEAK_MAC_PER_S, 4),
                     "hbm_staging_GBps": round(BC.ALGO_BYTES_PER_VERIFY * per_gpu_rate / 1e9, 2),
                     "note": "stage times (and the roofline kernel's launch time) from a second timed run with "
                             "stage-boundary events on the stream; value / ms_per_step from the run without them"},
        "verdicts_ok": bool(ok_local and (ok_all is None or ok_all)),
        "verdicts_check": "bitmap == known bits (valid except %d tampered records per GPU)%s" % (
            tamper_count(n), ", all %d shards' gathered bitmaps checked on every rank" % world if world > 1 else ""),
    }


def add_cpu_baseline(result, cb, c1=None):
    """Attach the libsodium CPU path timed on this box's host cores (rank 0, same run) to the line."""
    result["cpu_baseline"] = cb
    result["vs_cpu_baseline"] = round(result["value"] / cb["value"], 1) if cb.get("value") else None
    share = cb.get("per_gpu_share", {}).get("value")
    if share:
        result["vs_cpu_baseline_per_gpu_share"] = round(result["value"] / share, 1)
    if c1:
        result["cpu_baseline"]["config1_python_authenticate"] = c1
    return result


def feed_point_crossover(result):
    """The smallest host-buffer batch (of the measured sizes) whose verifies/s beat libsodium on all the
    host cores the cpu_baseline used, and the per-call drop-in against libsodium's own per-call loop:
    the numbers INTEGRATION.md §1 states (feed-point batching is required, not optional)."""
    cb = result.get("cpu_baseline", {}).get("value")
    lat = result.get("host_path", {}).get("batch_latency")
    if not cb or not lat:
        return
    sizes = sorted(int(k) for k in lat if k.isdigit())
    beat = [k for k in sizes if lat[str(k)]["verifies_per_s"] > cb]
    out = {"cpu_baseline_verifies_per_s": cb, "cores": result["cpu_baseline"].get("cores"),
           "smallest_batch_beating_cpu": beat[0] if beat else None,
           "per_size_verifies_per_s": {str(k): lat[str(k)]["verifies_per_s"] for k in sizes}}
    one = result.get("drop_in_per_call")
    c1 = result.get("cpu_baseline", {}).get("config1_python_authenticate")
    if one and c1:
        out["per_call_requests_per_s"] = {"gpu_unbatched": one["requests_per_s"], "libsodium_one_core": c1["requests_per_s"],
                                          "ratio": round(one["requests_per_s"] / c1["requests_per_s"], 3)}
    result["feed_point_crossover"] = out


class FileBarrier:
    """Host-side wait of ranks 1..N-1 while rank 0 runs a leg of its own (the CPU baseline, the
    single-process multi-GPU leg): a file per tag, polled with sleeps, so the waiting ranks spin
    neither a GPU collective nor a host core beside the leg being timed."""

    def __init__(self, world, rank):
        import tempfile
        self.world, self.rank = world, rank
        job = os.environ.get("PV_BENCH_JOB") or "%d_%s" % (os.getppid(), os.environ.get("MASTER_PORT", "0"))
        self.base = os.path.join(tempfile.gettempdir(), "pv_bench_%s" % job)
        self.made = []

    def release(self, tag):
        if self.rank == 0:
            p = "%s.%s.done" % (self.base, tag)
            with open(p, "w") as f:
                f.write("1")
            self.made.append(p)

    def wait(self, tag, timeout_s=1200):
        if self.rank == 0:
            return
        p = "%s.%s.done" % (self.base, tag)
        t0 = time.time()
        while not os.path.exists(p):
            if time.time() - t0 > timeout_s:
                raise TimeoutError("rank %d: rank 0's %s leg did not finish in %d s" % (self.rank, tag, timeout_s))
            time.sleep(0.05)

    def cleanup(self):
        for p in self.made:
            try:
                os.remove(p)
            except OSError:
                pass


def single_process_leg(blob, off, pks, want, world):
    """pv_verify_batch_multi_gpu from ONE process over the node's `world` GPUs (rank 0, while the other
    ranks wait): this rank's shard, host buffers in, sharded over every device with one in-process RCCL
    all-gather (the path a Plenum node process would use). Secondary, never `value`."""
    t0 = time.perf_counter()
    devs = _native.ensure_devices(range(world))
    init_s = time.perf_counter() - t0
    n = len(off) - 1
    _native.verify_sm_batch_multi(blob, off, pks, devs)  # warm: staging buffers sized on every device
    ts, ok = [], True
    for _ in range(3):
        t1 = time.perf_counter()
        got = _native.verify_sm_batch_multi(blob, off, pks, devs)
        ts.append(time.perf_counter() - t1)
        ok &= bool(np.array_equal(got, want))
    med = float(np.median(ts))
    try:
        clique = _native.multi_gpu_clique()
    except Exception as ex:
        clique = {"error": repr(ex)[:200]}
    return {"devices": list(devs), "requests": n, "verifies_per_s": round(n / med, 1), "seconds": round(med, 4),
            "init_devices_s": round(init_s, 2), "ok": ok, "rccl_clique": clique,
            "note": "pv_verify_batch_multi_gpu: host buffers, one worker thread per device (pinned staging + "
                    "H2D + verification on its own stream), one in-process ncclAllGather of the verdict words, "
                    "PCIe included; median of 3 calls"}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, cmd, poll_s=0.2):
    """Start n fresh rank processes of `cmd` (one per GPU), each with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT / PV_BENCH_JOB in its environment, relay rank 0's stdout
    and return 0 only if every rank exits 0. When a rank fails, the others (which would wait in a
    collective forever) are terminated by their exact PIDs. The caller never touches the GPU:
    this runs before the library is loaded (plain subprocess, never exec)."""
    import subprocess
    port = _free_port()
    job = "%d_%d" % (os.getpid(), port)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PV_BENCH_JOB=job)
        procs.append(subprocess.Popen(cmd, env=env, stdout=None if r == 0 else subprocess.DEVNULL))
    t0 = time.time()
    rc = 0
    live = list(range(n))
    last_note = t0
    while live:
        time.sleep(poll_s)
        for r in list(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.remove(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log("launcher: rank %d exited with %d after %.1f s; stopping the other ranks" % (r, code, time.time() - t0))
                for o in live:
                    procs[o].terminate()
        if rc and live:
            deadline = time.time() + 30
            while live and time.time() < deadline:
                live = [o for o in live if procs[o].poll() is None]
                time.sleep(poll_s)
            for o in live:
                procs[o].kill()
                procs[o].wait()
            live = []
        if live and time.time() - last_note > 60:
            last_note = time.time()
            log("launcher: %d of %d ranks still running (%.0f s)" % (len(live), n, time.time() - t0))
    return rc


def _rank_stub():
    """--rank-stub: what a rank saw (tests of the launcher; never touches the GPU)."""
    keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "PV_BENCH_JOB")
    out = os.environ.get("PV_BENCH_STUB_DIR")
    rec = {k: os.environ.get(k) for k in keys}
    rec["RANK"] = rec["RANK"] or "0"
    if out:
        with open(os.path.join(out, "rank%s.json" % rec["RANK"]), "w") as f:
            json.dump(rec, f)
    if os.environ.get("PV_BENCH_STUB_FAIL_RANK") == rec["RANK"]:
        sys.exit(3)
    if rec["RANK"] == "0":
        print(json.dumps({"stub": True, "world": int(rec["WORLD_SIZE"] or 1)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # untimed warm-up steps: after a cold start the 1M-request step settles from ~3.3 to ~2.75 ms
    # over its first ~12 steps (profiles/r02/step_warmup_trace.txt), so the default covers that
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--per-gpu", type=int, default=None,
                    help="requests per GPU (default: 1M at N = 1, configs[1]; ceil(64M / N) at N > 1, configs[4])")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sustain-s", type=float, default=2.0,
                    help="N = 1: seconds of back-to-back headline steps before the sustained_load sub-measurement "
                         "(0: skip it)")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-straus", action="store_true", help="skip the secondary Straus-path measurement")
    ap.add_argument("--no-config3", action="store_true", help="skip the configs[2] (2 % adversarial) leg")
    ap.add_argument("--dataset", default=None, help="npz from tools/nym_workload.py (profiling runs: no fork)")
    ap.add_argument("--no-ingress", action="store_true", help="skip the ingress / host-serialization measurements")
    ap.add_argument("--no-multisig", action="store_true", help="skip the configs[3] multi-signature measurement")
    ap.add_argument("--no-single-process", action="store_true",
                    help="N > 1: skip rank 0's pv_verify_batch_multi_gpu leg over every GPU of the node")
    ap.add_argument("--rank-stub", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    # one process per GPU: under a launcher (torch.distributed.run) WORLD_SIZE must equal --gpus;
    # without one, --gpus N > 1 starts the N ranks itself (fresh processes, before anything here
    # has loaded the library or touched a GPU) and relays rank 0's line
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != args.gpus:
        log("bench.py: WORLD_SIZE=%s but --gpus %d: refusing to report a line for the wrong GPU count"
            % (env_world, args.gpus))
        sys.exit(2)
    if env_world is None and args.gpus > 1:
        t0 = time.perf_counter()
        rc = spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:])
        log("launcher: %d ranks finished with rc %d in %.1f s" % (args.gpus, rc, time.perf_counter() - t0))
        sys.exit(rc)
    if args.gpus < 1:
        log("bench.py: --gpus must be >= 1")
        sys.exit(2)
    if args.rank_stub:
        _rank_stub()
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.per_gpu:
        n = args.per_gpu
    elif world == 1:
        n = 1 << 20
    else:  # configs[4]: the 64M-request batch sharded over the N GPUs (64-aligned shards)
        n = (CONFIG5_TOTAL + world * 64 - 1) // (world * 64) * 64
    phases = {}  # per-phase wall budget (stderr and the line's "phases_s")
    t0 = time.perf_counter()
    wire = None
    if args.dataset and os.path.exists(args.dataset):
        blob0, off, pks, lo = nym_workload.load(args.dataset)
        assert lo == rank * n and len(off) - 1 == n, "dataset does not match this rank's shard"
    elif world == 1 and not args.no_ingress:
        blob0, off, pks, *wire = nym_workload.generate_wire(rank * n, n)
    else:
        # configs[4] shards are 8-32M requests per rank: more signing workers per rank where the node
        # has the cores (16 is the per-GPU CPU share of a 1-GPU box; never above 64)
        cores = len(os.sched_getaffinity(0))
        workers = min(64, max(16, cores // world)) if world > 1 else None
        blob0, off, pks = nym_workload.generate(rank * n, n, workers=workers)
    gen_s = time.perf_counter() - t0
    phases["generation"] = gen_s
    log("rank %d: generated %d requests (%.1f MB) in %.1f s" % (rank, n, blob0.nbytes / 1e6, gen_s))
    # the headline batch carries must-reject records: ~0.1 % of messages with one flipped byte
    import adversarial_batch
    blob, tampered = adversarial_batch.tamper(blob0, off, tamper_count(n), seed=1000 + rank)
    c1 = None
    if world == 1 and wire and not args.no_cpu_baseline:
        t0 = time.perf_counter()
        c1 = config1_legs(wire)  # CPU leg, forked workers: before the device comes up
        phases["config1_cpu_leg"] = time.perf_counter() - t0
    multi = None
    if world == 1 and not args.no_multisig and not args.dataset:
        t0 = time.perf_counter()
        # before the device comes up (forked); ~1 % corrupted signatures among the 3 per request
        multi = nym_workload.generate_multisig(0, min(n, 1 << 20), 3, bad_frac=0.01, seed=4)
        log("rank %d: generated %d 3-signature requests in %.1f s" % (rank, min(n, 1 << 20), time.perf_counter() - t0))

    # the GPU runtime comes up only after the forked signing workers of the workload generator are
    # done: nothing forks once the device is initialised
    t0 = time.perf_counter()
    _native.ensure_device(local_rank)
    L = _native.lib()
    phases["pv_init"] = time.perf_counter() - t0
    hbm_ctx = hbm_in_use()  # the engine context: fixed-base comb, workspace, staging
    log("rank %d: device %d up (pv_init) in %.1f s" % (rank, local_rank, phases["pv_init"]))
    t0 = time.perf_counter()
    db = DeviceBatch(blob, off, pks)
    comm = Comm(world, rank, L) if world > 1 else None
    d_all = db._alloc(db.words * 8 * world) if world > 1 else None
    phases["upload"] = time.perf_counter() - t0
    log("rank %d: batch uploaded%s in %.1f s" % (rank, " and communicator up" if comm else "", phases["upload"]))

    def step():
        db.verify()
        if world > 1:
            _native.check(L.pv_allgather_verdicts(db.d_verdict, db.words, d_all, None), "pv_allgather_verdicts")

    def barrier_sync():
        _native.check(L.pv_sync(), "pv_sync")
        if comm:
            comm.barrier()

    def timed(steps, fn=step, stages=True):
        """steps timed passes bracketed by device sync + barrier; max over ranks; per-step stage
        times and chunks per step (stages=False: no stage-boundary events on the stream, whose extra
        queue packets would sit on the measured path; the headline's value comes from such a run)."""
        barrier_sync()
        L.pv_set_timing(1 if stages else 0)
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        barrier_sync()
        el = time.perf_counter() - t0
        if comm:
            el = comm.max_f64(el)
        if not stages:
            return el, None
        stage = (ctypes.c_double * len(_native.PV_STAGES))()
        launches = ctypes.c_int()
        _native.check(L.pv_stage_times(stage, len(_native.PV_STAGES), ctypes.byref(launches)), "pv_stage_times")
        L.pv_set_timing(0)
        timed.chunks = max(1, launches.value) / steps
        return el, {s: v / steps for s, v in zip(_native.PV_STAGES, list(stage))}

    # headline: the default (AUTO) path selection
    _native.set_path(_native.PV_PATH_AUTO)
    t0 = time.perf_counter()
    for _ in range(args.warmup):
        step()
    _native.check(L.pv_sync(), "pv_sync")
    phases["warmup"] = time.perf_counter() - t0
    log("rank %d: %d warm-up steps in %.1f s" % (rank, args.warmup, phases["warmup"]))
    t0 = time.perf_counter()
    elapsed, _ = timed(args.steps, stages=False)  # the headline: no stage events in the measured loop
    _, stage_ms = timed(args.steps)                # stage breakdown and the roofline kernel's launch time
    phases["timed"] = time.perf_counter() - t0
    log("rank %d: timed runs in %.1f s (headline %.3f s for %d steps)" % (rank, phases["timed"], elapsed, args.steps))
    chunks = timed.chunks
    path, nkeys = _native.last_path()
    comb = path == _native.PV_PATH_COMB

    # correctness of the timed work: the verdicts equal the batch's known bits (valid by
    # construction except the tampered records), on this rank and, gathered, on every rank
    want_local = np.ones(n, bool)
    want_local[tampered] = False
    ok_local = bool(np.array_equal(bits(db.verdict_words(), n), want_local))
    ok_all = None
    if world > 1:
        allw = db.verdict_words(d_all, db.words * world).reshape(world, db.words)
        ok_all = all(np.array_equal(bits(allw[r], n), expected_bits(n, r)) for r in range(world))

    result = assemble_result(world, n, args.steps, args.warmup, elapsed, stage_ms, chunks, comb, nkeys,
                             float(blob.nbytes) / n, ok_local, ok_all, per_gpu_fixed=bool(args.per_gpu),
                             fused=_native.comb_fused() and n / chunks > FUSED_MIN_REQ)
    if world == 1 and args.sustain_s > 0:
        # the same step under sustained load: the MI355X raises its clock over ~2 s of back-to-back
        # launches (1.74-1.80 GHz in the first step after idle, ~2.0 after 10 steps, ~2.2 after 2.5 s:
        # in-kernel s_memtime / s_memrealtime stamps, profiles/r06/clock/), so the headline's 5 warm-up +
        # 20 timed steps run below the clock a continuously loaded verifier holds. Reported beside the
        # headline, never as `value`
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.sustain_s:
            for _ in range(20):
                step()
            _native.check(L.pv_sync(), "pv_sync")
        els, _ = timed(args.steps, stages=False)
        result["sustained_load"] = {
            "value": round(n * world * args.steps / els, 1), "ms_per_step": round(1e3 * els / args.steps, 3),
            "steps": args.steps, "after_s": round(time.perf_counter() - t0 - els, 2),
            "verdicts_ok": bool(np.array_equal(bits(db.verdict_words(), n), want_local)),
            "note": "the headline step timed again after ~%.1f s of back-to-back steps (the clock a continuously "
                    "loaded GPU holds; the headline itself follows the driver's warm-up)" % args.sustain_s}
        phases["sustained_load"] = time.perf_counter() - t0
    hbm_run = hbm_in_use()
    if hbm_ctx and hbm_run:
        result["hbm"] = {"context_GB": round(hbm_ctx[0] / 1e9, 2), "with_batch_GB": round(hbm_run[0] / 1e9, 2),
                         "total_GB": round(hbm_run[1] / 1e9, 1),
                         "note": "device memory in use after pv_init (the engine context: fixed-base comb, "
                                 "workspace, staging) and after the batch upload and the timed steps "
                                 "(hipMemGetInfo, device-wide)"}
    if world > 1:
        result["rccl"] = rccl_summary(world, *comm.rccl_ranks())
    if world > 1 and not args.no_host_path:
        # SURVEY.md §8e host traffic: each rank's shard from host buffers (pv_verify_batch: pinned
        # staging pipelined with the H2D DMA, kernels, verdicts back), on up to configs[4]'s 8M-request
        # shard; max over ranks. Reported beside the device-resident headline, never as `value`.
        hs = min(n, CONFIG5_TOTAL // 8)
        ho = off[:hs + 1]
        err, hel, hv = None, 0.0, None
        try:  # a host-side limit must not cost the headline line; every rank still joins each collective
            _native.verify_sm_batch(blob[:int(ho[-1])], ho, pks[:hs])  # staging buffers sized
        except Exception as ex:
            err = ex
        barrier_sync()
        if err is None:
            try:
                t1 = time.perf_counter()
                hv = _native.verify_sm_batch(blob[:int(ho[-1])], ho, pks[:hs])
                hel = time.perf_counter() - t1
            except Exception as ex:
                err = ex
        hel = comm.max_f64(hel if err is None else 1e30)
        if hel >= 1e30:
            result["host_path"] = {"error": repr(err)[:200] if err else "failed on another rank"}
        else:
            result["host_path"] = {"verifies_per_s": round(hs * world / hel, 1), "requests_per_gpu": hs,
                                   "seconds": round(hel, 4), "ok": bool(np.array_equal(hv, want_local[:hs])),
                                   "note": "pv_verify_batch from host buffers on every rank at once, PCIe "
                                           "included, max over ranks"}
    if comb and not args.no_straus and world == 1:
        # the same batch forced through the per-request Straus path (what a batch of all-distinct
        # keys gets): reported beside the headline, never as `value`
        _native.set_path(_native.PV_PATH_STRAUS)
        step()
        ks = max(3, args.steps // 4)
        el2, _ = timed(ks, stages=False)
        _, st2 = timed(ks)
        _native.set_path(_native.PV_PATH_AUTO)
        ok2 = bool(np.array_equal(bits(db.verdict_words(), n), want_local))
        ach2 = BC.MAC_MSM_HALF_KERNEL * (n / timed.chunks) / (st2["msm"] / timed.chunks * 1e-3)
        result["straus_path"] = {
            "value": round(n * world * ks / el2, 1), "steps": ks, "ms_per_step": round(1e3 * el2 / ks, 3),
            "stages_ms": {s: round(v, 4) for s, v in st2.items()},
            "roofline": {"kernel": "pv_msm_kernel", "achieved": round(ach2 / 1e12, 3),
                         "frac": round(ach2 / BC.PEAK_MAC_PER_S, 4),
                         "algorithmic_mac_per_verify": round(BC.MAC_MSM_HALF_KERNEL),
                         "algorithm": "half-size split k = k1/k2 mod 8L, 32 windows of both scalars",
                         "traffic": pmc_traffic("pv_msm_kernel"),
                         "valu_issue_per_cu_cycle_pmc": pmc_valu_issue("pv_msm_kernel")},
            "verdicts_ok": ok2}
    c3 = None
    if rank == 0 and world == 1 and not args.no_config3:
        c3, c3_got, c3_batch = config3_leg(db, blob0, off, pks, max(3, args.steps), args.warmup, timed)
        result["config3"] = c3
    if rank == 0 and world == 1 and not args.no_host_path:
        # PCIe-inclusive host-buffer path (pv_verify_batch) on the headline batch itself
        t0 = time.perf_counter()
        result["host_path"] = host_path_leg(blob, off, pks, want_local)
        phases["host_path"] = time.perf_counter() - t0
        # latency of one host-buffer call at the batch sizes Plenum's feed points produce (a ZStack
        # client quota is 100 messages, a node quota 1,000): median of 200 calls (50
        # above 4,096 requests) after 20 untimed ones, AUTO
        # path (<= 4,096 requests: the latency path, pv_latency.hip). "warm" = the same with the 1,024
        # signers' keys in the node-side key cache (pv_key_cache_put, built before timing; the
        # headline never uses the cache)
        def latency_at(sizes):
            lat = {}
            for k in sizes:
                ko = off[:k + 1]
                kb, kp = blob[:int(ko[-1])], pks[:k]
                want_k = want_local[:k]
                for _ in range(20):  # warm-up: staging sized, clocks up
                    _native.verify_sm_batch(kb, ko, kp)
                ts, outs = [], []
                for _ in range(200 if k <= 4096 else 50):
                    t1 = time.perf_counter()
                    outs.append(_native.verify_sm_batch(kb, ko, kp))
                    ts.append(time.perf_counter() - t1)
                okk = all(bool(np.array_equal(o, want_k)) for o in outs)  # checked outside the timed calls
                med = float(np.median(ts))
                lat[str(k)] = {"median_ms": round(1e3 * med, 3), "verifies_per_s": round(k / med, 1),
                               "path": _native.last_path()[0], "ok": okk}
            return lat
        lat = latency_at((1, 2, 4, 8, 16, 32, 64, 100, 1000, 4096, 10000, 32768))

        # the device-buffer call at 2,049-4,096 requests: AUTO's latency-vs-keyed choice is made on
        # the device by the dedup kernels (no host key count); median of 20 enqueue+sync rounds
        def device_latency_at(sizes):
            out = {}
            for k in sizes:
                ko = off[:k + 1]
                kb = DeviceBatch(blob[:int(ko[-1])], ko, pks[:k])
                try:
                    kb.verify()
                    _native.check(L.pv_sync(), "pv_sync")
                    ts = []
                    for _ in range(20):
                        t1 = time.perf_counter()
                        kb.verify()
                        _native.check(L.pv_sync(), "pv_sync")
                        ts.append(time.perf_counter() - t1)
                    okk = bool(np.array_equal(bits(kb.verdict_words(), k), want_local[:k]))
                    out[str(k)] = {"median_ms": round(1e3 * float(np.median(ts)), 3), "path": _native.last_path()[0],
                                   "ok": okk}
                finally:
                    kb.free()
            out["note"] = ("pv_verify_batch_device on HBM-resident inputs (no PCIe), AUTO; path 2 = keyed "
                           "(the dedup counted >= 3 requests per key), 3 = latency")
            return out
        lat["device_call"] = device_latency_at((2048, 3072, 4096))
        # automatic admission (pv_key_cache_auto(2)), no manual put: a signer's key is cached behind
        # the second batch it appears in, so the repeat calls of latency_at run on cached tables
        _native.KeyCache.configure(2048)
        _native.KeyCache.auto(2)
        lat["auto_key_cache"] = latency_at((1, 100, 1000, 4096))
        lat["auto_key_cache"]["admitted"], lat["auto_key_cache"]["failed"] = _native.KeyCache.auto_stats()
        lat["auto_key_cache"]["note"] = ("pv_key_cache_auto(2): keys admitted on their 2nd appearance (the "
                                         "first warm-up call is the 1st), median of 200 calls; no pv_key_cache_put")
        _native.KeyCache.auto(0)
        _native.KeyCache.configure(0)
        t1 = time.perf_counter()
        _native.KeyCache.configure(2048)
        _native.KeyCache.put([p["vk"] for p in nym_workload._pool()])
        put_s = time.perf_counter() - t1
        lat["warm_key_cache"] = latency_at((1, 100, 1000, 4096, 10000, 32768))
        lat["warm_key_cache"]["put_1024_keys_s"] = round(put_s, 4)
        # the headline batch, device-resident, with the signers' tables in the node-side cache: the
        # keyed path reads them instead of building them (no key chain / table fill in the step).
        # Reported beside the headline, never as `value` (the headline builds every table per step)
        ks = args.steps
        for _ in range(max(1, args.warmup)):  # the headline's warm-up: the first steps after the puts run slower
            db.verify()
        elw, _ = timed(ks, stages=False)
        _, stw = timed(ks)
        result["warm_key_cache"] = {
            "value": round(n * ks / elw, 1), "unit": "verifies/s", "steps": ks,
            "ms_per_step": round(1e3 * elw / ks, 3), "stages_ms": {s: round(v, 4) for s, v in stw.items()},
            "comb_keys": _native.last_split()[1],
            "verdicts_ok": bool(np.array_equal(bits(db.verdict_words(), n), want_local)),
            # the same batch from host memory with the signers cached (what a node with a warm cache gets)
            "host_path": {k: v for k, v in host_path_leg(blob, off, pks, want_local).items() if k != "note"},
            "note": "configs[1] batch with the 1,024 signers in the node-side key cache (pv_key_cache_put "
                    "before timing; each cached signer also has radix-65536 rows, so its [k](-A) is 16 niels "
                    "additions inside [S]B's loop): dedup + per-request kernels only"}
        _native.KeyCache.configure(0)
        lat["note"] = ("host buffers in / verdict bits out, PCIe included; path 3 = latency (one workgroup "
                       "per request, limb-parallel), 1 = Straus; the tampered headline records are included")
        result["host_path"]["batch_latency"] = lat
        result["host_prep"] = {"workload_generation_s": round(gen_s, 2), "note": "serialize + sign, %d workers" % min(
            16, os.cpu_count() or 1)}
    if rank == 0 and world == 1 and wire and not args.no_host_path:
        # configs[0] through the unmodified per-call drop-in with the HIP engine (one launch per
        # signature), beside the libsodium leg of the same loop (cpu_baseline.config1_python_authenticate)
        t0 = time.perf_counter()
        result["drop_in_per_call"] = config1_python(wire, gpu=True)
        # the same loop with automatic key-cache admission on (a signer is cached on its 2nd signature):
        # the per-call singletons then take the cached-key latency kernel
        _native.KeyCache.configure(2048)
        _native.KeyCache.auto(2)
        try:
            keep = ("requests_per_s", "us_per_request", "accepted")
            adm0 = _native.KeyCache.auto_stats()[0]  # the counter is cumulative over the process
            first = config1_python(wire, gpu=True)  # admits: each signer's tables are built on its 2nd call
            warm = config1_python(wire, gpu=True)   # every signer cached: the cached-key latency kernel
            result["drop_in_per_call"]["auto_key_cache"] = {
                "admitting_pass": {k: v for k, v in first.items() if k in keep},
                "warm_pass": {k: v for k, v in warm.items() if k in keep},
                "admitted": _native.KeyCache.auto_stats()[0] - adm0,
                "note": "the same 10,000-request loop twice with pv_key_cache_auto(2): the first pass pays the "
                        "table builds (radix-256 + radix-65536 rows) of every signer it admits"}
        finally:
            _native.KeyCache.auto(0)
            _native.KeyCache.configure(0)
        phases["drop_in_per_call"] = time.perf_counter() - t0
    if multi is not None:
        result["multisig"] = multisig_leg(multi, min(n, 1 << 20), 3, max(3, args.steps // 4))
    if rank == 0 and world == 1 and wire:
        result["ingress"] = ingress_leg(n, blob0, off, wire, max(3, args.steps // 4), 1)
    # rank 0's own legs at N > 1 (the other ranks wait on a file, idle): the single-process multi-GPU
    # entry over every GPU of the node, then the CPU baseline on the node's host cores -- each in a
    # try/except so that a failure records an error and never costs the headline line
    fb = FileBarrier(world, rank) if world > 1 else None
    if rank == 0 and world > 1 and not args.no_single_process:
        t0 = time.perf_counter()
        try:
            result["single_process"] = single_process_leg(blob, off, pks, want_local, world)
        except Exception as ex:
            result["single_process"] = {"error": repr(ex)[:300]}
        phases["single_process_leg"] = time.perf_counter() - t0
    if rank == 0 and not args.no_cpu_baseline:
        t0 = time.perf_counter()
        try:
            cb, c3_want = cpu_baseline(blob0, off, pks, min(args.cpu_sample, n), args.cpu_seconds,
                                       config3=c3_batch if c3 else None)
            add_cpu_baseline(result, cb, c1)
            feed_point_crossover(result)
            if c3 is not None:
                c3["verdicts_match_libsodium"] = bool(np.array_equal(c3_got, c3_want))
                c3["mismatches"] = int((c3_got != c3_want).sum())
        except Exception as ex:
            result["cpu_baseline"] = {"error": repr(ex)[:300]}
        phases["cpu_baseline"] = time.perf_counter() - t0
    if fb:
        fb.release("rank0_legs")
        fb.wait("rank0_legs")
    if rank == 0:
        result["phases_s"] = {k: round(v, 2) for k, v in phases.items()}
        log("rank 0: phase budget (s): " + ", ".join("%s %.1f" % kv for kv in phases.items()))
        print(json.dumps(result), flush=True)
    db.free()
    if comm:
        comm.close()
    if fb:
        fb.cleanup()


if __name__ == "__main__":
    main()
