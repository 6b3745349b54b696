"""C5 pipeline driver (tools/c5_pipeline.py) at a small scale: k in {15, 17, 19, 21}, count +
exchange + export, sharded lookup + gather, sharded read graph + gather — 1 and 2 ranks on one GPU
(2 ranks through the library's host transport over gloo), every stage checked by rank 0 against
the single-process oracle over all ranks' data (--check)."""
import os
import socket
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ARGS = ["--scale", "0.0004", "--lr-cov", "20", "--check"]


def _worker(rank, world, port):
    import torch.distributed as dist
    import c5_pipeline
    os.environ["HGA_BENCH_BACKEND"] = "gloo"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        c5_pipeline.run(rank, world, c5_pipeline.parse(ARGS), group_ready=True)
    finally:
        dist.destroy_process_group()


def test_c5_pipeline_one_rank():
    import c5_pipeline
    out = c5_pipeline.run(0, 1, c5_pipeline.parse(ARGS))
    assert out["checked_against_oracle"] and set(out["per_k"]) == {15, 17, 19, 21}
    assert all(v["exported"] > 0 and v["connections"] > 0 for v in out["per_k"].values())


def test_c5_pipeline_two_ranks():
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(2, _port()), nprocs=2, start_method="spawn")
