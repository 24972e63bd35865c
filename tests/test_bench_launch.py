"""bench.py's multi-rank launcher: `python bench.py --gpus N` started as a
plain process runs N ranks itself (torch.distributed.run as a child) and rank 0's line carries
n_gpus = N; a rank whose WORLD_SIZE differs from --gpus refuses to report."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_launches_n_ranks(n):
    p = _run(["--gpus", str(n), "--launch-check"], _env(PPOX_DIST_BACKEND="gloo"))
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["config"]["parallelism"] == f"dp{n}"


def test_world_mismatch_refuses_to_report():
    p = _run(["--gpus", "2", "--launch-check"], _env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2
    assert p.stdout.strip() == ""
    assert "refusing to report" in p.stderr


def test_one_gpu_needs_no_launcher():
    p = _run(["--launch-check"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip())
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "single GPU"


@pytest.mark.gpu
def test_gpus_2_runs_the_workload_on_two_ranks():
    """The real bench at --gpus 2 on a tiny config, both ranks on the box's one GPU over gloo (RCCL
    refuses two ranks on one device; the driver's N-GPU runs use RCCL, one GPU per rank)."""
    p = _run(["--gpus", "2", "--envs", "64", "--nstep", "16", "--batch-size", "256", "--epochs", "1",
              "--steps", "1", "--warmup", "1", "--no-cpu-baseline"], _env(PPOX_DIST_BACKEND="gloo"), timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip())
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert out["config"]["parallelism"].startswith("dp2")
