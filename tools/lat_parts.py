"""Where a one-request host-buffer call's time goes above the kernel: the same records through the
Python wrapper (_native.verify_sm_batch), the CPython binding called directly on prepared arrays,
the ctypes entry point, and a C caller (microbench/zc_call). Development tool, run on the GPU box:
    python3 tools/lat_parts.py OUT_RECORDS_FILE
writes the records for microbench/zc_call and prints medians of 300 calls (us)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]

import nym_workload  # noqa: E402
from plenum_amd import _native  # noqa: E402


def med(fn, reps=300):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(1e6 * float(np.median(ts)), 1)


def main():
    blob, off, pks = nym_workload.generate(0, 100, workers=4)
    with open(sys.argv[1], "wb") as f:
        f.write(np.array([100, int(off[100])], np.uint64).tobytes())
        f.write(np.ascontiguousarray(off[:101], np.uint64).tobytes())
        f.write(np.ascontiguousarray(blob[:int(off[100])], np.uint8).tobytes())
        f.write(np.ascontiguousarray(pks[:100], np.uint8).tobytes())
    _native.ensure_device()
    out = {}
    for k in (1, 100):
        o = np.ascontiguousarray(off[:k + 1], np.uint64)
        b, p = np.ascontiguousarray(blob[:int(o[-1])], np.uint8), np.ascontiguousarray(pks[:k], np.uint8)
        bits = np.zeros((k + 7) // 8, np.uint8)
        fc = _native._fastcall()
        L = _native.lib()
        pb, po, pp, pv = (a.ctypes.data for a in (b, o, p, bits))
        out[str(k)] = {"wrapper": med(lambda: _native.verify_sm_batch(b, o, p)),
                       "fastcall_direct": med(lambda: fc.verify(b, o, p, bits)),
                       "ctypes_prebuilt_ptrs": med(lambda: L.pv_verify_batch(pb, po, k, pp, pv))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
