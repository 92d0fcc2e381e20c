"""Shape of one pv_comb_ab_kernel launch from its per-workgroup stamps (tools/clock_probe.py --dump):
workgroups in start order by groups of 256 (start range, duration, end), the first round's durations
by dispatch rank on the CU, and the number of running workgroups every 25 us.

    python tools/stamp_shape.py stamps.npz
"""
import sys

import numpy as np


def main():
    d = np.load(sys.argv[1])
    r0 = (d["r0"] - d["r0"].min()) / 100.0
    r1 = (d["r1"] - d["r0"].min()) / 100.0
    dur = r1 - r0
    b = np.arange(len(r0))
    o = np.argsort(r0)
    print("workgroups %d, span %.1f us, median duration %.1f us" % (len(r0), r1.max(), np.median(dur)))
    for q in range(0, len(r0), 256):
        sl = o[q:q + 256]
        print("start rank %4d: start %7.1f..%7.1f us, duration median %6.1f (min %6.1f, max %6.1f), last end %7.1f"
              % (q, r0[sl].min(), r0[sl].max(), np.median(dur[sl]), dur[sl].min(), dur[sl].max(), r1[sl].max()))
    first = r0 < 1.0
    print("first round (%d workgroups started at t = 0), duration by block index (= dispatch order on the CU):"
          % first.sum())
    for q in range(4):
        m = first & (b >= q * 256) & (b < (q + 1) * 256)
        if m.any():
            print("  blocks %4d-%4d: median %.1f us" % (q * 256, (q + 1) * 256 - 1, np.median(dur[m])))
    ts = np.arange(0, r1.max(), 25.0)
    conc = [int(((r0 <= t) & (r1 > t)).sum()) for t in ts]
    print("running workgroups every 25 us (1,024 = every slot):", conc)
    print("slot-busy fraction (workgroup time / (1,024 slots x span)): %.4f" % (dur.sum() / (1024.0 * r1.max())))


if __name__ == "__main__":
    main()
