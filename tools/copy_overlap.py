"""H2D copies against kernels in a rocprofv3 trace (rocpd SQLite output of --kernel-trace
--memory-copy-trace) of a host-buffer run (tools/host_path_probe.py): for the last `--calls` calls
(a call = the copies and kernels between two gaps of > `--gap-us` with nothing running), the span,
the time copies were active, the time kernels were active, and the time both were (the overlap the
pipelined sub-batches buy), plus the per-call event list with --events.

    python tools/copy_overlap.py TRACE_DB [--calls 2] [--events]
"""
import argparse
import sqlite3


def short(name):
    return str(name).replace("(anonymous namespace)::", "").split("(")[0]


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def intersect_len(a, b):
    """length of (union a) ∩ (union b)"""
    def merged(iv):
        out = []
        for s, e in sorted(iv):
            if out and s <= out[-1][1]:
                out[-1][1] = max(out[-1][1], e)
            else:
                out.append([s, e])
        return out
    A, B = merged(a), merged(b)
    i = j = tot = 0
    while i < len(A) and j < len(B):
        s, e = max(A[i][0], B[j][0]), min(A[i][1], B[j][1])
        if e > s:
            tot += e - s
        if A[i][1] < B[j][1]:
            i += 1
        else:
            j += 1
    return tot


def table_with(con, words):
    names = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    for w in words:
        for n in names:
            if w in n.lower():
                return n
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--calls", type=int, default=2)
    ap.add_argument("--gap-us", type=float, default=500.0)
    ap.add_argument("--events", action="store_true")
    ap.add_argument("--all-kernels", action="store_true", help="list every kernel, not only the step markers")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    kt = table_with(con, ("kernels",))
    ct = table_with(con, ("memory_copies", "memory_copy", "copies"))
    if not ct:
        names = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
        raise SystemExit("no copy table in %s: %s" % (a.db, names))
    ccols = [d[0] for d in con.execute("select * from %s limit 1" % ct).description]
    size_col = next((c for c in ("size", "bytes", "copy_bytes") if c in ccols), None)
    kind_col = next((c for c in ("name", "kind", "direction", "operation") if c in ccols), None)
    ev = []
    for r in con.execute("select name, start, end from %s" % kt):
        ev.append(("K", short(r[0]), int(r[1]), int(r[2]), 0))
    sel = "select start, end%s%s from %s" % ((", " + size_col) if size_col else "", (", " + kind_col) if kind_col else "", ct)
    for r in con.execute(sel):
        size = int(r[2]) if size_col else 0
        kind = r[3 if size_col else 2] if kind_col else "copy"
        ev.append(("C", str(kind), int(r[0]), int(r[1]), size))
    ev.sort(key=lambda x: x[2])
    # split into calls: each host-buffer call ends with its verdicts' device-to-host copy (else: at idle
    # gaps of > gap_us)
    calls, cur, end = [], [], None
    d2h = any(e[0] == "C" and "DEVICE_TO_HOST" in e[1] for e in ev)
    for e in ev:
        if not d2h and end is not None and e[2] - end > a.gap_us * 1e3:
            calls.append(cur)
            cur = []
        cur.append(e)
        end = e[3] if end is None else max(end, e[3])
        if d2h and e[0] == "C" and "DEVICE_TO_HOST" in e[1]:
            calls.append(cur)
            cur, end = [], None
    if cur:
        calls.append(cur)
    print("copy table %s columns %s" % (ct, ccols))
    for c in calls[-a.calls:]:
        t0 = min(e[2] for e in c)
        t1 = max(e[3] for e in c)
        ks = [(e[2], e[3]) for e in c if e[0] == "K"]
        cs = [(e[2], e[3]) for e in c if e[0] == "C"]
        cbytes = sum(e[4] for e in c if e[0] == "C")
        print("call: span %.1f us, copies active %.1f us (%d copies, %.1f MB), kernels active %.1f us (%d kernels), "
              "both %.1f us" % ((t1 - t0) / 1e3, union_len(cs) / 1e3, len(cs), cbytes / 1e6, union_len(ks) / 1e3, len(ks),
                                intersect_len(cs, ks) / 1e3))
        if a.events:
            for e in c:
                if e[0] == "C" or a.all_kernels or e[1].startswith(("pv_key_insert", "pv_encode", "pv_comb_a", "pv_unpermute")):
                    print("  %s %-34s %9.1f %9.1f %8.1f %s" % (e[0], e[1][:34], (e[2] - t0) / 1e3, (e[3] - t0) / 1e3,
                                                          (e[3] - e[2]) / 1e3, "%.1f MB" % (e[4] / 1e6) if e[4] else ""))


if __name__ == "__main__":
    main()
