"""Throughput of the engine on BASELINE config 3 (1M NYM requests, ~2 % adversarial: ~9k extra
distinct keys from the key-mutating classes) per arithmetic path, device-resident inputs.
Measurement helper (lives under tests/ because it uses the oracle as the checker; bench.py's headline is config 2):
    python tests/perf_config3.py [--steps K]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    from plenum_amd import _native
    from oracle.oracle import Oracle, cpu_verdicts
    from adversarial import inject
    import nym_workload
    from bench import DeviceBatch
    blob, off, pks = nym_workload.generate(0, 1 << 20)
    blob, pks, idx, _ = inject(blob, off, pks, 0.02, seed=3, oracle=Oracle())
    n = len(off) - 1
    nkeys = len(np.unique(pks, axis=0))
    _native.ensure_device()
    L = _native.lib()
    db = DeviceBatch(blob, off, pks)
    want = None
    out = {"config": "configs[2]: 1M NYM requests, 2 % adversarial", "requests": n, "distinct_keys": nkeys}
    for name, path in (("auto", _native.PV_PATH_AUTO), ("comb", _native.PV_PATH_COMB),
                       ("straus", _native.PV_PATH_STRAUS)):
        _native.set_path(path)
        db.verify()
        _native.check(L.pv_sync(), "sync")
        t0 = time.perf_counter()
        for _ in range(args.steps):
            db.verify()
        _native.check(L.pv_sync(), "sync")
        dt = (time.perf_counter() - t0) / args.steps
        got = np.unpackbits(db.verdict_words().view(np.uint8), bitorder="little")[:n].astype(bool)
        if want is None:
            want = cpu_verdicts(blob, off, pks)
        out[name] = {"verifies_per_s": round(n / dt), "ms_per_step": round(1e3 * dt, 3),
                     "path_taken": _native.last_path()[0], "bit_exact": bool(np.array_equal(got, want))}
    _native.set_path(_native.PV_PATH_AUTO)
    print(out, flush=True)


if __name__ == "__main__":
    main()
