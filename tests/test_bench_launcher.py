"""bench.py's own multi-GPU launcher (CPU only, no GPU touched): `python bench.py --gpus N` with no
WORLD_SIZE starts N fresh rank processes with the rank environment a torch.distributed.run agent
would give them, relays rank 0's line, and fails when a rank fails; WORLD_SIZE != --gpus is refused.
The rank body here is the hidden --rank-stub, which records the environment it saw and exits before
any workload, library or device work."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
RANK_KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "PV_BENCH_JOB")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in RANK_KEYS + ("LOCAL_WORLD_SIZE",)}
    env.update(extra)
    return env


def _run(args, env, timeout=120):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 8])
def test_launcher_spawns_ranks_with_rank_env(tmp_path, n):
    p = _run(["--gpus", str(n), "--rank-stub"], _env(PV_BENCH_STUB_DIR=str(tmp_path)))
    assert p.returncode == 0, p.stderr
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and json.loads(lines[0]) == {"stub": True, "world": n}  # rank 0's line only
    seen = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(n)]
    assert [s["RANK"] for s in seen] == [str(r) for r in range(n)]
    assert [s["LOCAL_RANK"] for s in seen] == [str(r) for r in range(n)]
    assert all(s["WORLD_SIZE"] == str(n) and s["MASTER_ADDR"] == "127.0.0.1" for s in seen)
    assert len({s["MASTER_PORT"] for s in seen}) == 1 and int(seen[0]["MASTER_PORT"]) > 0
    assert len({s["PV_BENCH_JOB"] for s in seen}) == 1 and seen[0]["PV_BENCH_JOB"]


def test_launcher_fails_when_a_rank_fails(tmp_path):
    p = _run(["--gpus", "4", "--rank-stub"], _env(PV_BENCH_STUB_DIR=str(tmp_path), PV_BENCH_STUB_FAIL_RANK="2"))
    assert p.returncode != 0
    assert "rank 2 exited with 3" in p.stderr


@pytest.mark.parametrize("world,gpus", [("3", "2"), ("1", "8"), ("8", "1")])
def test_world_size_mismatch_is_refused(world, gpus):
    p = _run(["--gpus", gpus, "--rank-stub"], _env(WORLD_SIZE=world, RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2
    assert "refusing" in p.stderr
    assert p.stdout.strip() == ""


def test_under_external_launcher_rank_runs_directly(tmp_path):
    """torch.distributed.run form: WORLD_SIZE == --gpus, this process IS the rank (no re-spawn)."""
    p = _run(["--gpus", "2", "--rank-stub"], _env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_PORT="29999",
                                                  PV_BENCH_STUB_DIR=str(tmp_path)))
    assert p.returncode == 0, p.stderr
    assert os.listdir(tmp_path) == ["rank1.json"]
    assert p.stdout.strip() == ""  # only rank 0 prints


def test_single_gpu_needs_no_launcher(tmp_path):
    p = _run(["--gpus", "1", "--rank-stub"], _env(PV_BENCH_STUB_DIR=str(tmp_path)))
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout.strip()) == {"stub": True, "world": 1}
