"""In-kernel clock of pv_comb_ab_kernel under sustained load (MI355X_MICROARCH.md "DVFS give-back"
item 6). Needs the diagnostic build (tools/build_variant.sh clock
-DPV_CLOCK_PROBE=1, selected with PLENUM_AMD_LIB=variants/clock/libplenum_verify.so): wave 0 of every
comb_ab workgroup stamps s_memtime / s_memrealtime at entry and exit.

    python tools/clock_probe.py [--dataset /tmp/nym_1m.npz] [--seconds 2.5] [--label base]

Runs the headline step (configs[1], 1M requests, device-resident) back to back for --seconds, then
reads the last launch's stamps: per workgroup clock = delta memtime / delta realtime x 100 MHz; prints
one JSON line (median / p10 / p90 over workgroups, the steps' wall ms, and the workgroup span).
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

import bench  # noqa: E402
import nym_workload  # noqa: E402
from plenum_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default=None)
    ap.add_argument("--seconds", type=float, default=2.5)
    ap.add_argument("--label", default="")
    ap.add_argument("--dump", default=None, help="also save the last launch's per-workgroup stamps (npz)")
    ap.add_argument("--ramp", action="store_true",
                    help="from an idle GPU: the stamps of steps 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64 run back to "
                         "back (a sync after each of those steps to read them): does the step time fall because "
                         "the clock rises, or at the same clock?")
    a = ap.parse_args()
    if a.dataset and os.path.exists(a.dataset):
        blob, off, pks, _ = nym_workload.load(a.dataset)
    else:
        blob, off, pks = nym_workload.generate(0, 1 << 20)
    _native.ensure_device(0)
    L = _native.lib()
    db = bench.DeviceBatch(blob, off, pks)
    if a.ramp:
        _native.check(L.pv_sync(), "pv_sync")
        time.sleep(2.0)  # idle first
        marks = {1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64}
        for step in range(1, 65):
            t1 = time.perf_counter()
            db.verify()
            if step in marks:
                _native.check(L.pv_sync(), "pv_sync")
                wall = time.perf_counter() - t1
                r = stamps(L, off)
                r.update({"label": a.label, "step": step, "wall_ms_incl_sync": round(1e3 * wall, 3)})
                print(json.dumps(r), flush=True)
        db.free()
        return
    for _ in range(5):
        db.verify()
    _native.check(L.pv_sync(), "pv_sync")
    steps, t0 = 0, time.perf_counter()
    while True:
        for _ in range(20):
            db.verify()
        steps += 20
        _native.check(L.pv_sync(), "pv_sync")
        el = time.perf_counter() - t0
        if el >= a.seconds:
            break
    out = {"label": a.label, "steps": steps, "seconds": round(el, 3), "ms_per_step": round(1e3 * el / steps, 4),
           "verifies_per_s": round((len(off) - 1) * steps / el, 1), "lib": os.path.basename(os.path.dirname(
               os.environ.get("PLENUM_AMD_LIB", "")) or "product")}
    out.update(stamps(L, off, a.dump))
    db.free()
    print(json.dumps(out), flush=True)


def stamps(L, off, dump=None):
    """Clock figures from the last comb_ab launch's stamps (diagnostic build), else an error entry.
    Also the launch's shape from the workgroups' start / end times (100 MHz ticks): span, the median
    workgroup time, how long the first and last 5 % of workgroups took to start and to end."""
    nblk = L.pv_test_clock_stamps(None, 0)
    if nblk <= 0:
        return {"error": "no stamps: not a PV_CLOCK_PROBE build"}
    grid = (len(off) - 1 + 255) // 256
    k = min(nblk, grid)
    buf = np.zeros(4 * k, np.uint64)
    got = L.pv_test_clock_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), k)
    st = buf[:4 * got].reshape(-1, 4).astype(np.float64)
    dt, dr = st[:, 1] - st[:, 0], st[:, 3] - st[:, 2]
    ok = (dr > 0) & (dt > 0)
    ghz = dt[ok] / dr[ok] * 0.1  # 100 MHz realtime ticks -> GHz
    span_us = (st[ok, 3].max() - st[ok, 2].min()) / 100.0
    r0 = st[ok, 2] - st[ok, 2].min()
    r1 = st[ok, 3] - st[ok, 2].min()
    if dump:
        np.savez(dump, t0=st[ok, 0], t1=st[ok, 1], r0=st[ok, 2], r1=st[ok, 3])
    shape = {"start_us_p5_p50_p95_max": [round(float(np.percentile(r0, q)) / 100.0, 1) for q in (5, 50, 95, 100)],
             "end_us_min_p5_p50_p95": [round(float(np.percentile(r1, q)) / 100.0, 1) for q in (0, 5, 50, 95)],
             # workgroup-time over (1,024 concurrent workgroup slots x span): 4 waves / SIMD x 4 SIMDs x 256 CUs
             # / 4 waves per workgroup
             "slot_busy_fraction": round(float((r1 - r0).sum()) / (1024.0 * float(r1.max())), 4)}
    return {"launch_shape": shape,"workgroups": int(ok.sum()), "clock_ghz_median": round(float(np.median(ghz)), 4),
            "clock_ghz_p10": round(float(np.percentile(ghz, 10)), 4),
            "clock_ghz_p90": round(float(np.percentile(ghz, 90)), 4),
            "wg_us_median": round(float(np.median(dr[ok])) / 100.0, 2),
            "wg_kcycles_median": round(float(np.median(dt[ok])) / 1e3, 1),
            "kernel_span_us_from_stamps": round(float(span_us), 1)}


if __name__ == "__main__":
    main()
