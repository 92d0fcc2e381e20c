"""Summarise rocprofv3 --pmc CSV passes into per-kernel, per-dispatch averages and the derived figures
the roofline uses. Usage: python tools/pmc_summary.py OUT.json DIR [DIR ...] [--requests N]

Derived (MI355X_MICROARCH.md §HBM / rocprofv3 notes):
  hbm_read_bytes  = FETCH_SIZE(KiB) * 1024        (raw; the gfx950 x2 correction is calibrated only for
                    wide coalesced streaming reads, so the corrected figure is kept as an upper bound)
  hbm_write_bytes = WRITE_SIZE(KiB) * 1024
  eff_clock_GHz   = GRBM_GUI_ACTIVE / 8 XCDs / kernel seconds
  valu_lane_instr_per_request = SQ_INSTS_VALU * 64 / requests
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0]


def load(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "*.csv")):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if "Counter_Name" not in row:
                        break
                    k = short(row["Kernel_Name"])
                    acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return acc, dur


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    requests = 1 << 20
    if "--requests" in sys.argv:
        requests = int(sys.argv[sys.argv.index("--requests") + 1])
    out, dirs = args[0], args[1:]
    acc, dur = load(dirs)
    summary = {"requests_per_dispatch": requests, "kernels": {}}
    for k, counters in acc.items():
        avg = {c: sum(v) / len(v) for c, v in counters.items()}
        secs = sorted(dur[k])[len(dur[k]) // 2]
        d = {"counters_per_dispatch": avg, "median_dispatch_s_under_pmc": secs}
        if "FETCH_SIZE" in avg:
            d["hbm_read_bytes"] = avg["FETCH_SIZE"] * 1024
            d["hbm_read_bytes_x2_upper"] = avg["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in avg:
            d["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in d and "hbm_write_bytes" in d:
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
            d["hbm_bytes_per_request"] = d["hbm_bytes_per_launch"] / requests
        if "GRBM_GUI_ACTIVE" in avg:
            d["eff_clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / secs / 1e9
        if "SQ_INSTS_VALU" in avg:
            d["valu_lane_instr_per_request"] = avg["SQ_INSTS_VALU"] * 64 / requests
        if "SQ_INSTS_SALU" in avg:
            d["salu_instr_per_request"] = avg["SQ_INSTS_SALU"] * 64 / requests
        if "SQ_WAVE_CYCLES" in avg and "SQ_WAVES" in avg:
            d["wave_cycles_per_wave"] = avg["SQ_WAVE_CYCLES"] / max(1.0, avg["SQ_WAVES"])
        if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
            d["valu_active_frac_of_wave_cycles"] = avg["SQ_ACTIVE_INST_VALU"] / max(1.0, avg["SQ_WAVE_CYCLES"])
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            d["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
        summary["kernels"][k] = d
    msm = summary["kernels"].get("pv_msm_kernel", {})
    summary["hbm_bytes_per_launch"] = msm.get("hbm_bytes_per_launch")
    with open(out, "w") as f:
        json.dump(summary, f, indent=1)
    for k, d in summary["kernels"].items():
        print(k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in d.items() if x != "counters_per_dispatch"})


if __name__ == "__main__":
    main()
