"""Host-buffer staging workers (indy-plenum_amd/csrc/copy_pool.h, compiled here with g++ exactly as the
library includes it): every device context has its own copy pool, so the per-device workers of
pv_verify_batch_multi_gpu stage their shards concurrently (the process-wide pool
serialised them); two callers of ONE pool take turns; the pinned-range registry that lets
pv_verify_batch skip the staging copy for pv_host_alloc / pv_host_register memory answers interior,
edge and foreign ranges exactly; the cache of released pinned blocks hands them out again by size. CPU
only."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "copy_pool_check.cpp")
BIN = os.path.join(HERE, "native", "copy_pool_check")


@pytest.fixture(scope="module")
def report():
    hdr = os.path.join(HERE, "..", "indy-plenum_amd", "csrc", "copy_pool.h")
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(SRC), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-o", BIN, SRC])
    out = subprocess.run([BIN], check=True, capture_output=True, text=True, timeout=60).stdout
    return json.loads(out)


def test_two_devices_stage_concurrently(report):
    c = report["concurrent_devices"]
    (a0, a1), (b0, b1) = c["w0"], c["w1"]
    # each device's tasks ran while the other device's were running
    assert a0 < b1 and b0 < a1, c
    overlap = min(a1, b1) - max(a0, b0)
    assert overlap > 0.5 * c["task_ms"], c
    # both shards staged in about the time of one (not two back to back)
    if report["threads_per_pool"] >= 2:
        assert c["wall_ms"] < 1.6 * (a1 - a0), c


def test_one_pool_takes_turns(report):
    s = report["same_pool"]
    (a0, a1), (b0, b1) = s["w0"], s["w1"]
    assert a1 <= b0 + 1.0 or b1 <= a0 + 1.0, s


def test_pool_sizes(report):
    assert report["pool_threads_8dev_256hw"] == 8
    assert report["pool_threads_1dev_4hw"] == 2


def test_pinned_registry(report):
    r = report["registry"]
    assert r["inner"] and r["whole"] and r["edge_end"] and r["other"]
    assert not r["past"] and not r["before"] and not r["other_past"]
    assert r["removed"] and r["gone"] and r["twice"]


def test_pinned_block_cache(report):
    """pv_host_free keeps released pinned blocks (up to a budget) for the next pv_host_alloc of a
    similar size: smallest fitting block, never one more than twice the request, oldest evicted."""
    assert all(report["pinned_cache"].values()), report["pinned_cache"]
