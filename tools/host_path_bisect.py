"""Development probe: host-path (pv_verify_batch) call times after a sequence of other engine uses, to
find what slows the pipelined DMA from the pinned arena (bench.py's cached host-path leg ran at half the
DMA rate of the same calls in a fresh process). Ops, run in order:
  host      3 alternating arena / pageable calls of the 1M batch (prints their times)
  cache     pv_key_cache configure(2048) + put the 1,024 signers
  nocache   configure(0)
  auto      configure(2048) + auto(2) + 120 latency-path calls (1 / 100 / 1,000 requests) + auto(0)
  lat       120 latency-path calls, as above, without the cache changes
  dev       20 device-resident verifications of the 1M batch (DeviceBatch)
    python tools/host_path_bisect.py --dataset /tmp/nym_1m.npz host cache host dev host
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]

import nym_workload  # noqa: E402
from plenum_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default=None)
    ap.add_argument("ops", nargs="+")
    a = ap.parse_args()
    if a.dataset and os.path.exists(a.dataset):
        blob, off, pks, _ = nym_workload.load(a.dataset)
    else:
        blob, off, pks = nym_workload.generate(0, 1 << 20)
    n = len(off) - 1
    _native.ensure_device(0)
    ab, ao, ak = _native.HostArena.batch(blob, off, pks)
    K = _native.KeyCache
    vks = [p["vk"] for p in nym_workload._pool()]

    def lat():
        for k in (1, 100, 1000):
            ko = off[:k + 1]
            for _ in range(40):
                _native.verify_sm_batch(blob[:int(ko[-1])], ko, pks[:k])

    for i, op in enumerate(a.ops):
        t0 = time.perf_counter()
        if op == "host":
            ts = {"arena": [], "pageable": []}
            for _ in range(3):
                for f, (b, o, k) in (("arena", (ab, ao, ak)), ("pageable", (blob, off, pks))):
                    t1 = time.perf_counter()
                    _native.verify_sm_batch(b, o, k)
                    ts[f].append(round(1e3 * (time.perf_counter() - t1), 2))
            print(json.dumps({"op": i, "host_ms": ts}), flush=True)
            print("-- op %d host done" % i, file=sys.stderr, flush=True)
            continue
        if op == "cache":
            K.configure(2048)
            K.put(vks)
        elif op == "nocache":
            K.configure(0)
        elif op == "auto":
            K.configure(2048)
            K.auto(2)
            lat()
            K.auto(0)
        elif op == "lat":
            lat()
        elif op == "dev":
            from bench import DeviceBatch
            db = DeviceBatch(blob, off, pks)
            for _ in range(20):
                db.verify()
            _native.check(_native.lib().pv_sync(), "pv_sync")
            db.free()
        else:
            raise SystemExit("unknown op " + op)
        print(json.dumps({"op": i, "name": op, "s": round(time.perf_counter() - t0, 3)}), flush=True)


if __name__ == "__main__":
    main()
