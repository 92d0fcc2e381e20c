"""Run the forced per-request Straus path on a synthetic NYM batch a few times (profiling driver:
rocprofv3 --kernel-trace / --pmc around it). Usage: python tools/straus_probe.py [N] [CALLS]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]

import nym_workload  # noqa: E402
from plenum_amd import _native  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    blob, off, pks = nym_workload.generate(0, n, workers=min(16, os.cpu_count() or 1))
    _native.ensure_device()
    _native.set_path(_native.PV_PATH_STRAUS)
    for _ in range(calls):
        v = _native.verify_sm_batch(blob, off, pks)
    print("requests", n, "accepted", int(np.count_nonzero(v)), flush=True)


if __name__ == "__main__":
    main()
