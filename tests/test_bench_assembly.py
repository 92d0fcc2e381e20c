"""bench.py's result assembly at N > 1, on CPU with stubbed measurements: the line
the driver's 8-GPU run prints carries the configs[4] workload, the roofline of the dominant kernel and
the libsodium CPU baseline timed in the same run; the host-side barrier rank 0's legs use releases the
waiting ranks."""
import os
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _stub_stages(ms_total):
    split = {"keys": 0.1, "prep": 0.5, "table": 0.7, "msm": 1.25, "encode": 0.18}
    scale = ms_total / sum(split.values())
    return {k: v * scale for k, v in split.items()}


@pytest.mark.parametrize("world", [2, 8])
def test_assemble_result_multi_gpu(world):
    n = (bench.CONFIG5_TOTAL + world * 64 - 1) // (world * 64) * 64
    chunks = n / (1 << 20)
    steps = 20
    elapsed = steps * 2.75e-3 * chunks  # ~2.75 ms per 1M chunk
    stage = {k: v * chunks for k, v in _stub_stages(2.72).items()}
    r = bench.assemble_result(world, n, steps, 5, elapsed, stage, chunks, True, 1024, 299.0, True, True)
    assert r["n_gpus"] == world and r["metric"] == bench.METRIC
    assert r["config"]["workload"].startswith("configs[4]: %d " % (n * world))
    assert r["config"]["requests_per_gpu"] == n and r["config"]["parallelism"] == "dp%d" % world
    assert r["scaling"] == "strong"
    assert abs(r["value"] - n * world * steps / elapsed) < 1
    rf = r["roofline"]
    assert rf["bound"] == "valu" and rf["kernel"] == "pv_comb_a_kernel"
    assert 0 < rf["frac"] < 1 and rf["peak"] > 30
    assert abs(rf["launch_ms"] - 1.25 * 2.72 / 2.73) < 0.01
    cb = {"value": 485000.0, "unit": "verifies/s", "cores": 16, "kind": "reference", "sample": "stub"}
    bench.add_cpu_baseline(r, cb, None)
    assert r["cpu_baseline"]["cores"] == 16 and r["cpu_baseline"]["kind"] == "reference"
    assert r["vs_cpu_baseline"] == round(r["value"] / 485000.0, 1)
    assert r["verdicts_ok"] is True
    # what RCCL itself reported on every rank (pv_comm_count), as bench.main puts it into the line
    r["rccl"] = bench.rccl_summary(world, [world] * world, list(range(world)))
    assert r["rccl"] == {"nranks": world, "rank": 0, "nranks_max_over_ranks": world,
                         "nranks_min_over_ranks": world, "user_ranks": list(range(world)), "ok": True}
    bad = bench.rccl_summary(world, [world] * (world - 1) + [1], list(range(world)))
    assert bad["nranks_min_over_ranks"] == 1 and bad["ok"] is False


def test_cpu_baseline_fields():
    """cpu_baseline carries the host's affinity-set count as `cores` and the per-GPU
    share beside it; the line states the ratio against both."""
    r = bench.assemble_result(1, 1 << 20, 20, 5, 20 * 2.7e-3, _stub_stages(2.7), 1, True, 1024, 299.0, True, None)
    cb = {"value": 5.9e6, "unit": "verifies/s", "cores": 224, "kind": "reference", "sample": "stub",
          "per_gpu_share": {"value": 4.8e5, "cores": 16}}
    bench.add_cpu_baseline(r, cb, None)
    assert r["vs_cpu_baseline"] == round(r["value"] / 5.9e6, 1)
    assert r["vs_cpu_baseline_per_gpu_share"] == round(r["value"] / 4.8e5, 1)


def test_assemble_result_single_gpu_straus():
    n = 1 << 20
    r = bench.assemble_result(1, n, 10, 5, 10 * 11e-3, _stub_stages(11.0), 1, False, 0, 299.0, True, None)
    assert r["config"]["workload"].startswith("configs[1]:")
    assert r["roofline"]["kernel"] == "pv_msm_kernel" and r["scaling"] == "weak"


def test_file_barrier_releases_waiting_rank(tmp_path, monkeypatch):
    monkeypatch.setenv("PV_BENCH_JOB", "test_%d" % os.getpid())
    r0, r1 = bench.FileBarrier(2, 0), bench.FileBarrier(2, 1)
    done = []
    t = threading.Thread(target=lambda: (r1.wait("legs", timeout_s=30), done.append(1)))
    t.start()
    time.sleep(0.1)
    assert not done
    r0.release("legs")
    t.join(10)
    assert done == [1]
    r0.wait("legs")  # rank 0 never waits on itself
    r0.cleanup()
    with pytest.raises(TimeoutError):
        bench.FileBarrier(2, 1).wait("never", timeout_s=0.05)
