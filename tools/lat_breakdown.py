"""Where the host-buffer latency of a small pv_verify_batch call goes (latency path, no stage events).

    python tools/lat_breakdown.py run [REPS [SIZES]]        # the calls (run under rocprofv3 --kernel-trace
                                                            #   --memory-copy-trace), prints median host times
    python tools/lat_breakdown.py analyze TRACE_DB          # per call: ops on the GPU, durations and gaps (us)
"""
import json
import os
import sqlite3
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]


def run(reps, sizes=(1, 100)):
    import nym_workload
    from plenum_amd import _native
    blob, off, pks = nym_workload.generate(0, max(sizes), workers=4)
    _native.ensure_device()
    _native.set_path(_native.PV_PATH_AUTO)
    out = {}
    for n in sizes:
        o = off[:n + 1]
        b, p = blob[:int(o[-1])], pks[:n]
        for _ in range(20):
            _native.verify_sm_batch(b, o, p)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            got = _native.verify_sm_batch(b, o, p)
            ts.append(time.perf_counter() - t0)
        out[str(n)] = {"median_us": round(1e6 * float(np.median(ts)), 1), "ok": bool(got.all())}
        time.sleep(0.05)  # a gap in the trace between the two sizes
    print(json.dumps(out), flush=True)


def analyze(db):
    con = sqlite3.connect(db)
    names = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    ops = []
    for r in con.execute("select name, start, end from kernels"):
        ops.append((int(r[1]), int(r[2]), r[0].split("(")[0][:40]))
    mc = next((t for t in ("memory_copies", "memory_copy") if t in names), None)
    if mc:
        cols = [d[0] for d in con.execute("select * from %s limit 1" % mc).description]
        kind = next((c for c in ("name", "direction", "kind") if c in cols), None)
        for r in con.execute("select %s, start, end from %s" % (kind or "'copy'", mc)):
            ops.append((int(r[1]), int(r[2]), "copy:" + str(r[0])[:30]))
    else:
        print("no memory-copy table; tables:", names)
    ops.sort()
    # calls: consecutive ops whose gaps are < 200 us; the two sizes are separated by a 50 ms sleep
    calls, cur = [], [ops[0]]
    for o in ops[1:]:
        if o[0] - cur[-1][1] > 40000:  # > 40 us idle = next call
            calls.append(cur)
            cur = [o]
        else:
            cur.append(o)
    calls.append(cur)
    # group by the time gap of > 10 ms (size switch)
    groups, g = [], [calls[0]]
    for c in calls[1:]:
        if c[0][0] - g[-1][-1][1] > 10_000_000:
            groups.append(g)
            g = [c]
        else:
            g.append(c)
    groups.append(g)
    for gi, g in enumerate(groups):
        sig = {}
        for c in g:
            key = tuple(o[2] for o in c)
            sig.setdefault(key, []).append(c)
        key, cs = max(sig.items(), key=lambda kv: len(kv[1]))
        print("== group %d: %d calls, most common op sequence (%d calls):" % (gi, len(g), len(cs)))
        t0s = [c[0][0] for c in cs]
        period = np.median(np.diff(t0s)) / 1e3 if len(t0s) > 1 else 0
        for j, name in enumerate(key):
            dur = np.median([c[j][1] - c[j][0] for c in cs]) / 1e3
            gap = np.median([c[j][0] - c[j - 1][1] for c in cs]) / 1e3 if j else 0.0
            print("   %-44s gap before %7.1f  dur %7.1f" % (name, gap, dur))
        span = np.median([c[-1][1] - c[0][0] for c in cs]) / 1e3
        print("   first op start -> last op end %.1f us; call period %.1f us" % (span, period))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 300,
            tuple(int(x) for x in sys.argv[3].split(",")) if len(sys.argv) > 3 else (1, 100))
    else:
        analyze(sys.argv[2])
