"""Phase timeline of one latency-path verification (measurement builds only).

Needs a library built with -DPV_LAT_TRACE (tools/build_variant.sh lattrace -DPV_LAT_TRACE), selected
with PLENUM_AMD_LIB. Verifies a 1-request batch `reps` times on the forced latency path and prints,
for the last call, block 0's s_memrealtime stamps (100 MHz) relative to wave 0's start, in us:
  wave 0: 0 start, 1 decompression done, 2 tables done, 3 past barrier 1, 4 loop done,
          5 past barrier 2, 6 verdict written
  waves 2, 3 (four-wave form): 14 start, 7 / 15 y-only chain done (lp_ydbl_chain)
  wave 0, four-wave zero-copy form: 16 kernel entry, 17 request slot copied into LDS (negative:
          before wave 0's start)
  wave 1: 8 start, 9 k ready, 12 split done, 13 k2 S mod L done, 18 recodings done (four-wave),
          10 digits and comb entries ready,
          11 [S]B / [k2](-R') + [s2]B done
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]

import nym_workload  # noqa: E402
from plenum_amd import _native  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    blob, off, pks = nym_workload.generate(0, 16, workers=1)
    _native.ensure_device()
    L = _native.lib()
    _native.set_path(_native.PV_PATH_LATENCY)
    o = off[:2]
    runs = []
    for _ in range(reps):
        got = _native.verify_sm_batch(blob[:int(o[-1])], o, pks[:1])
        buf = (ctypes.c_ulonglong * 20)()
        assert L.pv_debug_lat_trace(buf) == 0
        t = list(buf)
        runs.append({i: round((t[i] - t[0]) / 100.0, 2) for i in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18)})
        stats = {"lehmer_blocks": t[15] & 255, "block_quotients": (t[15] >> 8) & 255, "exact_steps": t[15] >> 16}
    med = {i: float(np.median([r[i] for r in runs])) for i in runs[0]}
    print(json.dumps({"lib": os.environ.get("PLENUM_AMD_LIB", "default"), "ok": bool(got[0]),
                      "median_us_from_wave0_start": med, "split_stats_last": stats}))


if __name__ == "__main__":
    main()
