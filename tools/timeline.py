"""Kernel timeline of the last K engine steps from a rocprofv3 kernel trace (rocpd SQLite output).

    python tools/timeline.py TRACE_DB [--steps K] [--first-kernel pv_key_insert_kernel]

A step starts at each launch of --first-kernel (the first kernel of a keyed chunk). Prints, per
kernel of the last K steps, its queue/stream, start and end relative to the step's start (us) and
its duration, so that overlap between the engine's streams (main, key stream, Straus side stream)
can be read directly.
"""
import argparse
import sqlite3


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--first-kernel", default="pv_key_insert")
    ap.add_argument("--summary", action="store_true",
                    help="one line per step of the whole trace: span and the main kernels' durations (us)")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cur = con.execute("select * from kernels limit 1")
    cols = [d[0] for d in cur.description]
    q = next((c for c in ("stream_id", "queue_id", "queue") if c in cols), None)
    sel = "select name, start, end%s from kernels order by start" % (", " + q if q else "")
    rows = [(short(r[0]), int(r[1]), int(r[2]), r[3] if q else "") for r in con.execute(sel)]
    starts = [i for i, r in enumerate(rows) if r[0].startswith(a.first_kernel)]  # also pv_key_insert_lds_kernel
    if not starts:
        raise SystemExit("no %s in the trace (columns: %s)" % (a.first_kernel, cols))
    if a.summary:
        keys = ("pv_key_insert", "pv_key_assign_kernel", "pv_key_scan_kernel", "pv_key_chain_lp_kernel", "pv_key_fill_kernel",
                "pv_comb_b_kernel", "pv_comb_a_kernel", "pv_comb_ab_kernel", "pv_msm_kernel", "pv_encode_kernel")
        print("row    span   " + " ".join("%8s" % k.replace("pv_", "").replace("_kernel", "")[:8] for k in keys)
              + "  comb_a_start")
        for j, s in enumerate(starts):
            nxt = starts[j + 1] if j + 1 < len(starts) else len(rows)
            t0 = rows[s][1]
            span = (max(r[2] for r in rows[s:nxt]) - t0) / 1e3
            dur = {}
            ca = 0.0
            for name, st, en, _ in rows[s:nxt]:
                for k in keys:
                    if name.endswith(k) or name.startswith(k) or name.startswith("void " + k):
                        dur[k] = dur.get(k, 0.0) + (en - st) / 1e3
                if "pv_comb_a_kernel" in name or "pv_comb_ab_kernel" in name:
                    ca = (st - t0) / 1e3
            print("%5d %7.1f " % (s, span) + " ".join("%8.1f" % dur.get(k, 0.0) for k in keys) + "  %8.1f" % ca)
        return
    for s in starts[-a.steps:]:
        t0 = rows[s][1]
        nxt = next((i for i in starts if i > s), len(rows))
        end = max(r[2] for r in rows[s:nxt])
        print("== step at row %d: %.1f us from first kernel start to last kernel end" % (s, (end - t0) / 1e3))
        for name, st, en, qq in rows[s:nxt]:
            print("  %-28s %-6s %9.1f %9.1f %8.1f" % (name, qq, (st - t0) / 1e3, (en - t0) / 1e3, (en - st) / 1e3))


if __name__ == "__main__":
    main()
