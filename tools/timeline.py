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
    ap.add_argument("--first-kernel", default="pv_key_insert_kernel")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cur = con.execute("select * from kernels limit 1")
    cols = [d[0] for d in cur.description]
    q = next((c for c in ("stream_id", "queue_id", "queue") if c in cols), None)
    sel = "select name, start, end%s from kernels order by start" % (", " + q if q else "")
    rows = [(short(r[0]), int(r[1]), int(r[2]), r[3] if q else "") for r in con.execute(sel)]
    starts = [i for i, r in enumerate(rows) if r[0] == a.first_kernel]
    if not starts:
        raise SystemExit("no %s in the trace (columns: %s)" % (a.first_kernel, cols))
    for s in starts[-a.steps:]:
        t0 = rows[s][1]
        nxt = next((i for i in starts if i > s), len(rows))
        end = max(r[2] for r in rows[s:nxt])
        print("== step at row %d: %.1f us from first kernel start to last kernel end" % (s, (end - t0) / 1e3))
        for name, st, en, qq in rows[s:nxt]:
            print("  %-28s %-6s %9.1f %9.1f %8.1f" % (name, qq, (st - t0) / 1e3, (en - t0) / 1e3, (en - st) / 1e3))


if __name__ == "__main__":
    main()
