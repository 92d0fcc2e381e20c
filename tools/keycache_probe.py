"""The headline batch device-resident, with the signers' comb tables built inside every step (fresh) or
read from the node-side key cache (cached): per-step time and stage times, one JSON line (development
tool for the cached-comb A/B and its PMC passes; one mode per process so that rocprofv3's per-kernel
figures belong to one mode).

    python tools/keycache_probe.py --dataset npz --mode fresh|cached [--steps 10] [--warmup 5]
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
from bench import DeviceBatch, bits  # noqa: E402
from plenum_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default=None)
    ap.add_argument("--mode", choices=("fresh", "cached"), default="fresh")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cap", type=int, default=2048)
    a = ap.parse_args()
    if a.dataset and os.path.exists(a.dataset):
        blob, off, pks, _ = nym_workload.load(a.dataset)
    else:
        blob, off, pks = nym_workload.generate(0, 1 << 20)
    n = len(off) - 1
    _native.ensure_device(0)
    L = _native.lib()
    put_s = None
    if a.mode == "cached":
        t0 = time.perf_counter()
        _native.KeyCache.configure(a.cap)
        _native.KeyCache.put([p["vk"] for p in nym_workload._pool()])
        put_s = time.perf_counter() - t0
    db = DeviceBatch(blob, off, pks)
    for _ in range(a.warmup):
        db.verify()
    _native.check(L.pv_sync(), "pv_sync")
    t0 = time.perf_counter()
    for _ in range(a.steps):
        db.verify()
    _native.check(L.pv_sync(), "pv_sync")
    el = time.perf_counter() - t0
    L.pv_set_timing(1)
    for _ in range(a.steps):
        db.verify()
    _native.check(L.pv_sync(), "pv_sync")
    st = (ctypes.c_double * len(_native.PV_STAGES))()
    launches = ctypes.c_int()
    _native.check(L.pv_stage_times(st, len(_native.PV_STAGES), ctypes.byref(launches)), "pv_stage_times")
    L.pv_set_timing(0)
    ok = bool(bits(db.verdict_words(), n).all())
    split = _native.last_split()
    db.free()
    print(json.dumps({"mode": a.mode, "requests": n, "ms_per_step": round(1e3 * el / a.steps, 4),
                      "verifies_per_s": round(n * a.steps / el, 1), "put_s": put_s,
                      "stages_ms": {s: round(v / a.steps, 4) for s, v in zip(_native.PV_STAGES, list(st))},
                      "split": list(split), "all_valid": ok}), flush=True)


if __name__ == "__main__":
    main()
