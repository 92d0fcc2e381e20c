"""Host-fed throughput probe (development tool): pv_verify_batch on host buffers at several batch
sizes, median of `reps` calls after one warm-up, pageable numpy inputs and (when the library has
pv_host_alloc) inputs built in the library's pinned arena. One JSON line per measurement.

    python tools/host_path_probe.py [--dataset npz] [--sizes 262144,1048576] [--reps 5]
"""
import argparse
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
    ap.add_argument("--dataset", default=None)
    ap.add_argument("--sizes", default="262144,1048576")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-arena", action="store_true")
    ap.add_argument("--cache", type=int, default=0, help="key cache capacity; the 1,024 signers are put before timing")
    args = ap.parse_args()
    sizes = [int(x) for x in args.sizes.split(",")]
    nmax = max(sizes)
    t0 = time.perf_counter()
    if args.dataset and os.path.exists(args.dataset):
        blob, off, pks, _ = nym_workload.load(args.dataset)
    else:
        blob, off, pks = nym_workload.generate(0, nmax)
    print(json.dumps({"generated": len(off) - 1, "s": round(time.perf_counter() - t0, 2)}), flush=True)
    _native.ensure_device(0)
    if args.cache:
        _native.KeyCache.configure(args.cache)
        _native.KeyCache.put([p["vk"] for p in nym_workload._pool()])
    arena = None
    if not args.no_arena and hasattr(_native, "HostArena"):
        arena = _native.HostArena
    for k in sizes:
        ko = off[:k + 1]
        kb, kp = blob[:int(ko[-1])], pks[:k]
        forms = [("pageable", kb, ko, kp)]
        if arena is not None:
            forms.append(("arena",) + arena.batch(kb, ko, kp))
        ts = {f[0]: [] for f in forms}
        oks = {f[0]: True for f in forms}
        for name, b, o, p in forms:
            _native.verify_sm_batch(b, o, p)
        # the forms alternate call by call, so a shared-PCIe slowdown hits both alike
        for _ in range(args.reps):
            for name, b, o, p in forms:
                t1 = time.perf_counter()
                v = _native.verify_sm_batch(b, o, p)
                ts[name].append(time.perf_counter() - t1)
                oks[name] &= bool(v.all())
        for name, _, _, _ in forms:
            med = float(np.median(ts[name]))
            print(json.dumps({"requests": k, "form": name, "median_ms": round(med * 1e3, 3),
                              "min_ms": round(min(ts[name]) * 1e3, 3), "verifies_per_s": round(k / med, 1),
                              "ok": oks[name], "blob_MB": round(int(ko[-1]) / 1e6, 1),
                              "all_ms": [round(t * 1e3, 2) for t in ts[name]]}), flush=True)


if __name__ == "__main__":
    main()
