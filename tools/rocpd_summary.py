"""Summarise rocprofv3 (ROCm 7.2, rocpd SQLite output) runs of bench.py into committed evidence.

    python tools/rocpd_summary.py OUTDIR TRACE_DB [PMC_DB ...] [--requests N]

Writes OUTDIR/kernel_stats.csv (the --stats view: calls, total/avg/min/max ns per kernel; gated-off
launches of the path the chunk did not take are counted separately as `gated_calls`) and
OUTDIR/pmc_summary.json (per kernel, per real dispatch: every counter summed over its hardware
instances, averaged over dispatches, plus derived figures):
  hbm_read_bytes  = FETCH_SIZE (KiB) * 1024      raw, as the counter reports it
  hbm_read_bytes_x2 = 2 x that                   MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of the
                                                  bytes of a wide coalesced 16-B/lane stream on gfx950
  hbm_write_bytes = WRITE_SIZE (KiB) * 1024
  hbm_bytes_per_launch_corrected = hbm_read_bytes_x2 + hbm_write_bytes   (bench roofline.traffic)
  eff_clock_GHz   = GRBM_GUI_ACTIVE / 8 XCDs / dispatch seconds
  valu_instr_per_request = SQ_INSTS_VALU * 64 / requests   (wave-instructions x 64 lanes)
A dispatch shorter than GATED_NS is a launch the device-side path gate turned into a no-op.
"""
import csv
import json
import os
import sqlite3
import sys
from collections import defaultdict

GATED_NS = 20000


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def kernel_stats(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, duration from kernels").fetchall()
    per = defaultdict(list)
    for name, dur in rows:
        per[short(name)].append(int(dur))
    total = sum(sum(v) for v in per.values()) or 1
    out = []
    for k, v in per.items():
        real = [d for d in v if d >= GATED_NS] or v
        out.append({"Name": k, "Calls": len(real), "GatedCalls": len(v) - len(real),
                    "TotalDurationNs": sum(real), "AverageNs": round(sum(real) / len(real), 1),
                    "Percentage": round(100.0 * sum(v) / total, 3), "MinNs": min(real), "MaxNs": max(real)})
    out.sort(key=lambda r: -r["TotalDurationNs"])
    return out


def pmc(dbs):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for db in dbs:
        con = sqlite3.connect(db)
        q = ("select kernel_name, dispatch_id, counter_name, sum(value), max(duration) from counters_collection "
             "group by dispatch_id, counter_name")
        seen = set()
        for name, disp, ctr, val, d in con.execute(q):
            k = short(name)
            if d < GATED_NS:
                continue
            acc[k][ctr].append(float(val))
            if (db, disp) not in seen:
                seen.add((db, disp))
                dur[k].append(d * 1e-9)
    return acc, dur


def main():
    argv = sys.argv[1:]
    if "--requests" in argv:  # drop the option and its value
        i = argv.index("--requests")
        argv = argv[:i] + argv[i + 2:]
    args = [a for a in argv if not a.startswith("--")]
    requests = 1 << 20
    if "--requests" in sys.argv:
        requests = int(sys.argv[sys.argv.index("--requests") + 1])
    outdir, trace, pmcs = args[0], args[1], args[2:]
    os.makedirs(outdir, exist_ok=True)
    stats = kernel_stats(trace)
    with open(os.path.join(outdir, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(stats[0].keys()))
        w.writeheader()
        w.writerows(stats)
    for r in stats:
        print("%-24s calls=%4d gated=%3d avg=%10.1f us  min=%10.1f max=%10.1f" % (
            r["Name"], r["Calls"], r["GatedCalls"], r["AverageNs"] / 1e3, r["MinNs"] / 1e3, r["MaxNs"] / 1e3))
    if not pmcs:
        return
    acc, dur = pmc(pmcs)
    summary = {"requests_per_dispatch": requests, "kernels": {}}
    for k, counters in acc.items():
        avg = {c: sum(v) / len(v) for c, v in counters.items()}
        secs = sorted(dur[k])[len(dur[k]) // 2] if dur[k] else None
        d = {"counters_per_dispatch": avg, "median_dispatch_s_under_pmc": secs}
        if "FETCH_SIZE" in avg:
            d["hbm_read_bytes"] = avg["FETCH_SIZE"] * 1024
            d["hbm_read_bytes_x2"] = avg["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in avg:
            d["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in d and "hbm_write_bytes" in d:
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
            # the guide's gfx950 correction (FETCH_SIZE x 2 for 16-B/lane streaming reads) + writes:
            # the figure the bench line reports as roofline.traffic
            d["hbm_bytes_per_launch_corrected"] = d["hbm_read_bytes_x2"] + d["hbm_write_bytes"]
            d["hbm_bytes_per_request"] = d["hbm_bytes_per_launch"] / requests
        if "GRBM_GUI_ACTIVE" in avg and secs:
            d["eff_clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / secs / 1e9
        if "SQ_INSTS_VALU" in avg:
            d["valu_instr_per_request"] = avg["SQ_INSTS_VALU"] * 64 / requests
        if "SQ_WAVE_CYCLES" in avg and "SQ_WAVES" in avg:
            d["wave_cycles_per_wave"] = avg["SQ_WAVE_CYCLES"] / max(1.0, avg["SQ_WAVES"])
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            d["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
        summary["kernels"][k] = d
    with open(os.path.join(outdir, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    for k, d in summary["kernels"].items():
        print(k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in d.items() if x != "counters_per_dispatch"})


if __name__ == "__main__":
    main()
