"""Development probe: NUMA placement of the pinned arena (pv_host_alloc) against the GPU's node, and
the H2D rate of pipelined host calls from it. One JSON line per process.
    python tools/numa_probe.py [--dataset npz]"""
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tools")]
import nym_workload  # noqa: E402
from plenum_amd import _native  # noqa: E402

libc = ctypes.CDLL(None, use_errno=True)


def page_nodes(addr, nbytes, samples=256):
    """NUMA node of `samples` pages spread over [addr, addr + nbytes) (move_pages with nodes=NULL)."""
    pg = os.sysconf("SC_PAGE_SIZE")
    pages = (ctypes.c_void_p * samples)(*[(addr + (nbytes * i // samples)) & ~(pg - 1) for i in range(samples)])
    status = (ctypes.c_int * samples)()
    rc = libc.syscall(279, 0, ctypes.c_ulong(samples), pages, None, status, 0)
    if rc != 0:
        return {"error": ctypes.get_errno()}
    h = {}
    for s in status:
        h[int(s)] = h.get(int(s), 0) + 1
    return h


def cpu_node(cpu):
    for p in glob.glob("/sys/devices/system/cpu/cpu%d/node*" % cpu):
        return int(p.rsplit("node", 1)[1])
    return -1


def main():
    ds = sys.argv[2] if len(sys.argv) > 2 and sys.argv[1] == "--dataset" else None
    blob, off, pks = (nym_workload.load(ds)[:3] if ds and os.path.exists(ds) else nym_workload.generate(0, 1 << 20))
    _native.ensure_device(0)
    L = _native.lib()
    bus = ctypes.create_string_buffer(64)
    gpu_node = None
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        dev = ctypes.c_int()
        hip.hipGetDevice(ctypes.byref(dev))
        if hip.hipDeviceGetPCIBusId(bus, 64, dev.value) == 0:
            bdf = bus.value.decode().lower()
            with open("/sys/bus/pci/devices/%s/numa_node" % bdf) as f:
                gpu_node = int(f.read())
    except Exception as ex:  # noqa: BLE001
        gpu_node = "err %s" % ex
    cpu = libc.sched_getcpu()
    ab, ao, ak = _native.HostArena.batch(blob, off, pks)
    ts = {"arena": [], "pageable": []}
    for b, o, k in ((ab, ao, ak), (blob, off, pks)):
        _native.verify_sm_batch(b, o, k)
    for _ in range(3):
        for f, (b, o, k) in (("arena", (ab, ao, ak)), ("pageable", (blob, off, pks))):
            t1 = time.perf_counter()
            _native.verify_sm_batch(b, o, k)
            ts[f].append(round(1e3 * (time.perf_counter() - t1), 2))
    print(json.dumps({"gpu_bdf": bus.value.decode(), "gpu_node": gpu_node, "cpu": cpu, "cpu_node": cpu_node(cpu),
                      "affinity_nodes": sorted({cpu_node(c) for c in os.sched_getaffinity(0)}),
                      "arena_blob_nodes": page_nodes(ab.ctypes.data, ab.nbytes),
                      "numpy_blob_nodes": page_nodes(blob.ctypes.data, blob.nbytes),
                      "host_ms": ts}), flush=True)


if __name__ == "__main__":
    main()
