"""bench.py's multi-GPU launcher (CPU, no GPU call): `python bench.py --gpus N` without torchrun
starts N rank processes itself (torch.distributed.run on 127.0.0.1) and rank 0 reports n_gpus = N;
a world size that differs from --gpus is an error (non-zero exit), never a silent single-rank run.
HGA_BENCH_DRYRUN=1 stops each rank right after the process group is up (gloo), before any GPU call."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(HGA_BENCH_BACKEND="gloo", HGA_BENCH_DRYRUN="1", **kw)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "1"], env=_env(), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 only
    out = json.loads(lines[0])
    assert out["dryrun"] and out["n_gpus"] == n


def test_world_size_mismatch_fails():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr


def test_one_gpu_is_one_rank():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0   # torchrun with 2 ranks but --gpus 1
