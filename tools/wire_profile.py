"""cProfile of authenticate_wire_packed on the bench's wire workload (1M NYM requests, 1,024 signers):
where the host time of the end-to-end ingress goes. python tools/wire_profile.py [n]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]

import nym_workload  # noqa: E402
from plenum_amd import _native, wire  # noqa: E402
from plenum_amd.client_authn import CoreAuthNr  # noqa: E402
from plenum_amd.req_authenticator import ReqAuthenticator  # noqa: E402


def make_ra(pool):
    core = CoreAuthNr(["1"], ["105"], [], state=None)
    for p in pool:
        core.addIdr(p["did"], p["abbr"])
    ra = ReqAuthenticator()
    ra.register_authenticator(core)
    return ra


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    _, _, _, wblob, woff, _, _ = nym_workload.generate_wire(0, n, workers=16)
    pool = nym_workload._pool()
    _native.ensure_device()
    threads = min(16, len(os.sched_getaffinity(0)))
    wire.authenticate_wire_packed(make_ra(pool), wblob[:int(woff[4096])], woff[:4097], threads)
    for _ in range(2):
        tm = {}
        t0 = time.perf_counter()
        wire.authenticate_wire_packed(make_ra(pool), wblob, woff, threads, timings=tm)
        dt = time.perf_counter() - t0
        print("req/s %.0f" % (n / dt), {k: round(v, 4) for k, v in tm.items()}, flush=True)
    ra = make_ra(pool)
    prof = cProfile.Profile()
    prof.enable()
    wire.authenticate_wire_packed(ra, wblob, woff, threads)
    prof.disable()
    pstats.Stats(prof).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
