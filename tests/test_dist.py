"""world_size > 1 counting protocol (hga_dist.OwnerExchange) on the CPU with gloo.

Each rank counts a contiguous shard of every file's reads; after the owner
exchange the gathered histogram and export must equal the single-process oracle pipeline over
all reads (JellyfishOccurrenceReader.cpp:63-135 semantics)."""
import random
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import hga_dist
import oracle

K = 11
THR = oracle.THRESHOLDS


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_streams(seed=7, n_reads=600, L=3000):
    rng = random.Random(seed)
    g = "".join(rng.choice("ACGT") for _ in range(L))
    h = list(g)
    for i in range(0, L, 37):
        h[i] = "ACGT"[("ACGT".index(h[i]) + 1) % 4]
    h = "".join(h)
    out = []
    for src in (g, h):
        reads = []
        for _ in range(n_reads):
            s = rng.randrange(0, L - 60)
            r = list(src[s: s + rng.randrange(20, 60)])
            if rng.random() < 0.3:
                r[rng.randrange(len(r))] = rng.choice("ACGTN")
            reads.append("".join(r))
        out.append(("\n".join(reads) + "\n").encode())
    return out


def _worker(rank, world, port, lower, upper, out_path, packed=True):
    from dist_engine_oracle import OracleEngine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        streams = make_streams()
        shards = [hga_dist.shard_reads(s, rank, world) for s in streams]
        ex = hga_dist.OwnerExchange(OracleEngine(shards, K, packed))
        ex.count(2)
        hist = ex.spec_hist(THR)
        keys, flags = ex.select(lower, upper)
        n, d = ex.select_counts(lower, upper)
        if rank == 0:
            np.savez(out_path, hist=hist, keys=keys, flags=flags, n=n, d=d)
    finally:
        dist.destroy_process_group()


def _run(world, tmp_path, lower=3, upper=40, packed=True):
    out = str(tmp_path / f"dist_{world}_{packed}.npz")
    mp.start_processes(_worker, args=(world, _free_port(), lower, upper, out, packed), nprocs=world,
                       start_method="spawn")
    return np.load(out)


@pytest.mark.parametrize("world,packed", [(2, True), (3, True), (2, False)])
def test_owner_exchange_matches_single_process(world, packed, tmp_path):
    r = _run(world, tmp_path, packed=packed)
    ref = oracle.count_pipeline(make_streams(), K, 3, 40)
    assert np.array_equal(r["hist"], ref["hist"])
    assert np.array_equal(r["keys"], ref["selected"])
    assert int(r["n"]) == len(ref["selected"]) and int(r["d"]) == ref["n_discr"]
    assert int(r["flags"].sum()) == ref["n_discr"]


def test_splitters_and_shards():
    for k in (1, 5, 19, 32):
        for n in (1, 2, 3, 8):
            s = hga_dist.owner_splitters(k, n)
            assert len(s) == n - 1 and np.all(np.diff(s.astype(object)) >= 0) if n > 2 else True
            assert all(int(x) < 4 ** k for x in s)
    seq = b"ACGT\nAC\n\nGGGTTT\nA\n"
    for w in (1, 2, 3, 5):
        parts = [hga_dist.shard_reads(seq, r, w) for r in range(w)]
        assert b"".join(parts) == seq
        assert all(p == b"" or p.endswith(b"\n") for p in parts)
