"""Profiling probe for the device ingress front end (no forked workers, so it can run under
rocprofv3): signs N synthetic NYM requests in-process, then runs bench.ingress_leg.
    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/ingress_probe.py [N]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]

import bench  # noqa: E402
import nym_workload  # noqa: E402
from plenum_amd import _native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
blob, off, pks, *wire = nym_workload.generate(0, n, workers=1, wire=True)
_native.ensure_device(0)
print(json.dumps(bench.ingress_leg(n, blob, off, wire, 5, 1)), flush=True)
