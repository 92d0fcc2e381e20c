"""Latency of one verification call at Plenum's feed-point batch sizes, per arithmetic path.

For each batch size n and path: the host-buffer call pv_verify_batch (pinned staging, H2D, kernels,
D2H: what a node's ingress would call) as the median of `reps` calls, and the device time of the
verification itself (pv_stage_times over the same calls). Verdicts are checked against the batch's
known bits (valid NYM requests, one tampered record per 16). Prints one JSON object.

    python tools/latency_probe.py [--sizes 1,100,1000] [--reps 20] [--paths latency,straus]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]

import nym_workload  # noqa: E402
from plenum_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,10,100,1000,2048,4096")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--paths", default="latency,straus,auto")
    ap.add_argument("--warm", action="store_true",
                    help="also measure the latency path with the 1,024 signer keys in the node-side key cache")
    args = ap.parse_args()
    sizes = [int(x) for x in args.sizes.split(",")]
    nmax = max(sizes)
    blob, off, pks = nym_workload.generate(0, nmax, workers=min(16, os.cpu_count() or 1))
    blob = blob.copy()
    bad = np.arange(7, nmax, 16)
    for i in bad:
        blob[int(off[i]) + 100] ^= 0x04
    want = np.ones(nmax, bool)
    want[bad] = False
    _native.ensure_device()
    L = _native.lib()
    out = {"requests_signers": 1024, "tampered_every": 16, "results": {}}
    runs = [(p, False) for p in args.paths.split(",")] + ([("latency", True)] if args.warm else [])
    for pname, warm in runs:
        if warm:
            t0 = time.perf_counter()
            _native.KeyCache.configure(2048)
            _native.KeyCache.put([p["vk"] for p in nym_workload._pool()])
            out["key_cache_put_1024_keys_s"] = round(time.perf_counter() - t0, 3)
        mode = getattr(_native, "PV_PATH_" + pname.upper())
        _native.set_path(mode)
        res = {}
        for n in sizes:
            o = off[:n + 1]
            b, p = blob[:int(o[-1])], pks[:n]
            got = _native.verify_sm_batch(b, o, p)  # warm-up
            ok = bool(np.array_equal(got, want[:n]))
            ts = []
            L.pv_set_timing(1)
            for _ in range(args.reps):
                t0 = time.perf_counter()
                got = _native.verify_sm_batch(b, o, p)
                ts.append(time.perf_counter() - t0)
                ok &= bool(np.array_equal(got, want[:n]))
            st = (ctypes.c_double * 5)()
            launches = ctypes.c_int()
            _native.check(L.pv_stage_times(st, 5, ctypes.byref(launches)), "pv_stage_times")
            L.pv_set_timing(0)
            dev_ms = sum(st) / max(1, launches.value)
            path, _ = _native.last_path()
            res[str(n)] = {"median_ms": round(1e3 * float(np.median(ts)), 4), "min_ms": round(1e3 * min(ts), 4),
                           "device_ms": round(dev_ms, 4), "path_taken": path, "ok": ok,
                           "verifies_per_s": round(n / float(np.median(ts)), 1)}
            print(pname + ("_warm" if warm else ""), n, res[str(n)], file=sys.stderr, flush=True)
        out["results"][pname + ("_warm_key_cache" if warm else "")] = res
        if warm:
            _native.KeyCache.configure(0)
    _native.set_path(_native.PV_PATH_AUTO)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
