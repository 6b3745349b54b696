"""GPU side of the owner exchange (exchange.hip through the C ABI, hga_dist.py).

(a) G ranks simulated in one process: G contexts count contiguous shards with min 1, partition
    their rows by owner into torch device buffers, owner o merges the slices addressed to it;
    the union of owner rows must equal the oracle's merged rows over all reads with the `--bc`
    drop (run_jellyfish.sh:3-6), and the per-owner histograms / exports must add up to the
    single-context results.
(b) The product path in the C ABI (hga_comm_init_host + hga_count_exchange, set up by
    hga_dist.OwnerExchange) in 2 and 3 processes sharing cuda:0, the library's transport hook over
    gloo (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's bench): every rank's
    global rows, dumps, histogram, export and stats equal the single-process oracle."""
import socket

import numpy as np
import pytest
import torch

import hga
import hga_dist
import oracle
from test_dist import make_streams

THR = oracle.THRESHOLDS
pytestmark = pytest.mark.gpu


def _sim(streams, k, G, lower, upper, min_c=2):
    F = len(streams)
    dev = torch.device("cuda:0")
    ctxs = [hga.Ctx(0) for _ in range(G)]
    spl = hga_dist.owner_splitters(k, G)
    sends = []
    for r, c in enumerate(ctxs):
        c.count_begin(k, F)
        for f, s in enumerate(streams):
            c.count_add(f, hga_dist.shard_reads(s, r, G))
        c.count_run(1)
        rows = c.count_stats().distinct_rows
        kb = torch.empty(rows, dtype=torch.int64, device=dev)
        cb = torch.empty(rows * F, dtype=torch.int32, device=dev)
        per = c.count_partition(spl, kb.data_ptr(), cb.data_ptr()).astype(np.int64)
        assert int(per.sum()) == rows
        off = np.concatenate([[0], np.cumsum(per)])
        sends.append((kb, cb, off))
    keys, counts, hist, sel, disc = [], [], [], [], 0
    for o, c in enumerate(ctxs):
        rk = torch.cat([kb[off[o]:off[o + 1]] for kb, _, off in sends])
        rc = torch.cat([cb[off[o] * F:off[o + 1] * F] for _, cb, off in sends])
        torch.cuda.synchronize()
        c.count_merge(rk.data_ptr(), rc.data_ptr(), len(rk), min_c)
        kk, cc = c.rows()
        if len(kk):
            lo = 0 if o == 0 else int(spl[o - 1])
            hi = 1 << 64 if o == G - 1 else int(spl[o])
            assert lo <= int(kk.min()) and int(kk.max()) < hi
        keys.append(kk)
        counts.append(cc)
        hist.append(c.spec_hist(THR) if len(kk) else np.zeros((0, 3), np.int64))
        s, f, d = c.select(lower, upper)
        sel.append(s)
        disc += d
    for c in ctxs:
        c.close()
    acc = {}
    for h in hist:
        for t, tot, n in h:
            acc[(int(t), int(tot))] = acc.get((int(t), int(tot)), 0) + int(n)
    H = np.array([[t, tot, acc[(t, tot)]] for t, tot in sorted(acc)], np.int64).reshape(-1, 3)
    return np.concatenate(keys), np.concatenate(counts), H, np.concatenate(sel), disc


@pytest.mark.parametrize("k,G", [(11, 2), (11, 3), (19, 4), (32, 5), (3, 8)])
def test_partition_merge_equals_oracle(k, G):
    streams = make_streams()
    keys, counts, H, sel, disc = _sim(streams, k, G, 3, 40)
    ref = oracle.count_pipeline(streams, k, 3, 40)
    assert np.array_equal(keys, ref["keys"])
    assert np.array_equal(counts, ref["counts"])
    assert np.array_equal(H, ref["hist"])
    assert np.array_equal(sel, ref["selected"]) and disc == ref["n_discr"]


def test_partition_merge_min_counts_and_empty_owner():
    streams = make_streams(seed=3, n_reads=200)
    for min_c in (1, 3):
        keys, counts, _, _, _ = _sim(streams, 9, 3, 2, 10, min_c)
        dumps = [oracle.count_stream(s, 9, min_c) for s in streams]
        rk, rc = oracle.merge(dumps)
        assert np.array_equal(keys, rk) and np.array_equal(counts, rc)
    # a world larger than the distinct codes of k=1 leaves owners empty
    keys, counts, _, _, _ = _sim(streams, 1, 6, 1, 10 ** 9)
    rk, rc = oracle.merge([oracle.count_stream(s, 1, 2) for s in streams])
    assert np.array_equal(keys, rk) and np.array_equal(counts, rc)


def _worker(rank, world, port, out_path, k, envs=None, big=False, root=-1):
    import os
    import torch.distributed as dist
    if envs:   # this rank's exchange test hooks (count.hip / exchange.hip)
        os.environ.update(envs[rank])
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ctx = hga.Ctx(0)
    try:
        streams = make_streams(seed=3, n_reads=100000, L=1500000) if big else make_streams()
        ctx.count_begin(k, len(streams))
        for f, s in enumerate(streams):
            ctx.count_add(f, hga_dist.shard_reads(s, rank, world))
        ex = hga_dist.OwnerExchange(ctx)
        assert ctx.comm_info() == (rank, world)
        if root >= 0:
            ctx.comm_set_root(root)
        ex.count(2)
        hist = ex.spec_hist(THR)
        keys, flags = ex.select(3, 40)
        n, d = ex.select_counts(3, 40)
        rk, rc = ctx.rows()
        d0 = ctx.dump(0)
        st = ctx.count_stats()
        np.savez(out_path + f".{rank}.npz", hist=hist, keys=keys, flags=flags, n=n, d=d, rk=rk, rc=rc, d0k=d0[0],
                 d0c=d0[1], inst=st.instances, rows=st.distinct_rows)
    finally:
        ctx.close()
        dist.destroy_process_group()


GEN = {"HGA_XB_GENERIC": "1"}           # sender bins its rows itself (kx_xb_hist / kx_xb_scatter)
WIDE = {"HGA_XB_WIDE": "1", "HGA_FB_MIN": "10"}   # owner table with u64 keys
EMIT = {"HGA_FB_MIN": "10"}             # count buckets fine enough for the count kernel's emission


def _gen(r):
    return {"HGA_XB_GENERIC": "1", "HGA_XB_R": str(r)}


@pytest.mark.parametrize("world,k,envs,big,one_pass", [
    (2, 13, None, False, False), (3, 27, None, False, False), (3, 19, (WIDE,) * 3, False, False),
    (2, 13, (EMIT, EMIT), False, False), (3, 27, (EMIT,) * 3, False, False),
    (2, 13, (_gen(10), _gen(12)), False, False),                  # senders at different resolutions
    (3, 19, (EMIT, _gen(10), _gen(13)), False, False),            # count-kernel emission next to generic senders
    (2, 19, (EMIT, EMIT), True, False), (2, 19, (GEN, GEN), True, False),
    (1, 19, (_gen(10),), True, False), (1, 19, (_gen(10),), True, True)])   # multi-pass / overflowing buckets
def test_count_exchange_processes(tmp_path, monkeypatch, world, k, envs, big, one_pass):
    """The hash-bucket exchange (exchange.hip kx_xb_*): senders' pieces grouped by the count kernel
    (count.hip XbEmit) or binned by the sender (GEN), owners merge every sender's runs of their
    buckets at the coarsest resolution any sender used; `big` (2.1 M rows at min 1) at 1024 owner
    buckets puts about 2 K pieces in each, so the owner merge takes two passes per bucket (and with
    HGA_MB_ONE_PASS a first attempt in one pass overflows its table and is retried)."""
    import torch.multiprocessing as mp
    if one_pass:
        monkeypatch.setenv("HGA_MB_ONE_PASS", "1")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "d")
    mp.start_processes(_worker, args=(world, port, out, k, envs, big), nprocs=world, start_method="spawn")
    streams = make_streams(seed=3, n_reads=100000, L=1500000) if big else make_streams()
    ref = oracle.count_pipeline(streams, k, 3, 40)
    inst = sum(oracle.count_instances(x, k) for x in streams)
    for rank in range(world):
        r = np.load(out + f".{rank}.npz")
        assert np.array_equal(r["hist"], ref["hist"])
        assert np.array_equal(r["keys"], ref["selected"])
        assert int(r["flags"].sum()) == ref["n_discr"]
        assert int(r["n"]) == len(ref["selected"]) and int(r["d"]) == ref["n_discr"]
        assert np.array_equal(r["rk"], ref["keys"]) and np.array_equal(r["rc"], ref["counts"])
        assert np.array_equal(r["d0k"], ref["dumps"][0][0]) and np.array_equal(r["d0c"], ref["dumps"][0][1])
        assert int(r["inst"]) == inst and int(r["rows"]) == len(ref["keys"])


def _sim_packed(streams, k, G, min_c):
    """Packed exchange simulated in one process: pieces per owner, owner merges its slices."""
    F = len(streams)
    dev = torch.device("cuda:0")
    ctxs = [hga.Ctx(0) for _ in range(G)]
    spl = hga_dist.owner_splitters(k, G)
    sends = []
    for r, c in enumerate(ctxs):
        c.count_begin(k, F)
        for f, s in enumerate(streams):
            c.count_add(f, hga_dist.shard_reads(s, r, G))
        c.count_run(1)
        assert c.count_pack_bits() > 0
        rows = c.count_stats().distinct_rows
        cap = max(rows // 4, 1)   # deliberately small: exercises the retry
        buf = torch.empty(cap, dtype=torch.int64, device=dev)
        per, tot = c.count_partition_packed(spl, buf.data_ptr(), cap)
        if tot > cap:
            buf = torch.empty(tot, dtype=torch.int64, device=dev)
            per, tot = c.count_partition_packed(spl, buf.data_ptr(), tot)
        per = per.astype(np.int64)
        assert int(per.sum()) == tot >= rows
        sends.append((buf, np.concatenate([[0], np.cumsum(per)])))
    keys, counts = [], []
    for o, c in enumerate(ctxs):
        rb = torch.cat([b[off[o]:off[o + 1]] for b, off in sends])
        torch.cuda.synchronize()
        c.count_merge_packed(rb.data_ptr(), len(rb), min_c)
        kk, cc = c.rows()
        keys.append(kk)
        counts.append(cc)
    for c in ctxs:
        c.close()
    return np.concatenate(keys), np.concatenate(counts)


@pytest.mark.parametrize("k,G,min_c", [(11, 3, 2), (13, 2, 2), (19, 4, 2), (27, 2, 1), (27, 5, 3)])
def test_packed_partition_merge_equals_oracle(k, G, min_c):
    base = make_streams(seed=k, n_reads=300)
    # repeated reads push counts past 2^5 - 1 at k = 27 (5 count bits per file): rows split into pieces
    streams = [s * 40 for s in base] if k == 27 else base
    keys, counts = _sim_packed(streams, k, G, min_c)
    rk, rc = oracle.merge([oracle.count_stream(s, k, min_c) for s in streams])
    assert np.array_equal(keys, rk)
    assert np.array_equal(counts, rc)
    if k == 27:
        assert int(counts.max()) > 31


def _mix_inv(h, k):
    """Inverse of kmer_dev.hpp's Mix on 2k bits (the owner merge bins pieces by its top bits)."""
    n = 2 * k
    mask = np.uint64((1 << n) - 1)
    s = np.uint64((n + 1) // 2)
    c1 = 0x9E3779C07F4A7C15   # kmer_dev.hpp kMixC1
    c1i = pow(c1, -1, 1 << 64)
    h = h ^ (h >> s)
    return (h * np.uint64(c1i)) & mask


@pytest.mark.parametrize("skew,one_pass", [(False, False), (True, False), (True, True)])
def test_merge_packed_many_pieces(skew, one_pass, monkeypatch):
    """Owner merge at scale against a numpy group-by: 3 M pieces (many buckets, repeated keys,
    split rows); with skew, a twelfth of them in ONE bucket of the merge's mix binning, so that
    bucket is summed in several passes over its LDS table; one_pass forces a first attempt in one
    pass per bucket, whose table overflow must be detected and retried."""
    if one_pass:
        monkeypatch.setenv("HGA_MB_ONE_PASS", "1")
    k, F, min_c = 19, 2, 2
    rng = np.random.default_rng(7)
    n = 3_000_000
    n_keys = 1_200_000
    if skew:
        mb = 12   # the merge's bucket bits for this n (about 1024 pieces per bucket)
        low = rng.integers(0, 1 << (2 * k - mb), n_keys // 12, dtype=np.uint64)
        hot = _mix_inv((np.uint64(5) << np.uint64(2 * k - mb)) | low, k)
        keys = np.concatenate([rng.integers(0, 1 << (2 * k), n_keys - len(hot), dtype=np.uint64), hot])
    else:
        keys = rng.integers(0, 1 << (2 * k), n_keys, dtype=np.uint64)
    pk = keys[rng.integers(0, n_keys, n)]
    cb = (64 - 2 * k) // F
    cnt = rng.integers(0, 4, (n, F)).astype(np.uint64)
    cnt[rng.random(n) < 0.001, 0] = (1 << cb) - 1          # saturated pieces of split rows
    cnt[cnt.sum(axis=1) == 0, 1] = 1
    pieces = pk.copy()
    for f in range(F):
        pieces |= cnt[:, f] << np.uint64(2 * k + f * cb)
    u, inv = np.unique(pk, return_inverse=True)
    tot = np.zeros((len(u), F), np.int64)
    for f in range(F):
        np.add.at(tot[:, f], inv, cnt[:, f].astype(np.int64))
    tot[tot < min_c] = 0
    keep = tot.any(axis=1)
    c = hga.Ctx(0)
    try:
        c.count_begin(k, F)
        assert c.count_pack_bits() == cb
        buf = torch.from_numpy(pieces.view(np.int64)).to("cuda:0")
        torch.cuda.synchronize()
        c.count_merge_packed(buf.data_ptr(), n, min_c)
        kk, cc = c.rows()
    finally:
        c.close()
    assert np.array_equal(kk, u[keep])
    assert np.array_equal(cc.reshape(-1, F).astype(np.int64), tot[keep])


def _lk_worker(rank, world, port, out_path):
    import torch.distributed as dist
    from test_dist import lookup_case
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ctx = hga.Ctx(0)
    try:
        hga_dist.attach(ctx)
        reads, sdk = lookup_case()
        a, b = len(reads) * rank // world, len(reads) * (rank + 1) // world
        mine = reads[a:b]
        ctx.lookup_load(13, sdk)
        ctx.lookup_set_reads(b"".join(mine), np.cumsum([0] + [len(r) for r in mine]).astype(np.uint64), 1 + a)
        ctx.lookup_run()
        ctx.lookup_gather()
        got = ctx.lookup_fetch()
        sz = ctx.lookup_sizes()
        cat = (np.arange(len(reads)) % 3).astype(np.int32)
        ctx.connections_run(pivots=np.arange(1 + a, 1 + b, dtype=np.uint32), min_score=2, categories=cat)
        n = ctx.connections_gather()
        x, y, s, g = (np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(n, np.uint64), np.zeros(n, np.uint8))
        hga.lib().hga_connections_fetch(ctx._h, x.ctypes.data_as(hga._u32p), y.ctypes.data_as(hga._u32p),
                                        s.ctypes.data_as(hga._u64p), g.ctypes.data_as(hga._u8p))
        np.savez(out_path + f".{rank}.npz", x=x, y=y, s=s, g=g, n_reads=sz.n_reads, hits=sz.hits, **got)
        ctx.lookup_run()   # back to this rank's own reads
        assert ctx.lookup_sizes().n_reads == len(mine)
    finally:
        ctx.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_lookup_gather_and_connections(tmp_path, world):
    """SURVEY.md §8(e) row 2 through the C ABI: each rank looks up its contiguous ReadID range,
    hga_lookup_gather builds the whole input's index on every rank, each rank's pivots are connected
    over it and hga_connections_gather joins them: equal to the single-process oracle
    (construct_indices, ReadClusteringEngine.cpp:234-299; get_connections, :301-333)."""
    import torch.multiprocessing as mp
    from test_dist import _free_port, lookup_case
    out = str(tmp_path / "lk")
    mp.start_processes(_lk_worker, args=(world, _free_port(), out), nprocs=world, start_method="spawn")
    reads, sdk = lookup_case()
    offs = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    ref = oracle.construct_indices(b"".join(reads), offs, 13, sdk, first_read_id=1)
    cat = (np.arange(len(reads)) % 3).astype(np.int32)
    rx, ry, rs, rg = oracle.connections(ref, min_score=2, categories=cat)
    for rank in range(world):
        r = np.load(out + f".{rank}.npz")
        assert int(r["n_reads"]) == len(reads) and int(r["hits"]) == len(ref["hit_kid"])
        for name in ref:
            assert np.array_equal(r[name], ref[name]), name
        assert np.array_equal(r["x"], rx) and np.array_equal(r["y"], ry)
        assert np.array_equal(r["s"], rs) and np.array_equal(r["g"], rg)


@pytest.mark.parametrize("world,root,envs", [(2, 1, None), (3, 0, (EMIT, _gen(10), EMIT))])
def test_gathered_lists_to_one_root(tmp_path, world, root, envs):
    """hga_comm_set_root (the export and the dumps to one writer, as the reference's
    single export pass, JellyfishOccurrenceReader.cpp:110-135): after the exchange, select / rows / dump
    deliver the whole list on the root only — equal to the oracle there — and empty lists elsewhere; the
    histogram and the global counts stay on every rank."""
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "d")
    mp.start_processes(_worker, args=(world, port, out, 13, envs, False, root), nprocs=world, start_method="spawn")
    ref = oracle.count_pipeline(make_streams(), 13, 3, 40)
    for rank in range(world):
        r = np.load(out + f".{rank}.npz")
        assert np.array_equal(r["hist"], ref["hist"])
        assert int(r["rows"]) == len(ref["keys"])
        if rank == root:
            assert np.array_equal(r["keys"], ref["selected"]) and int(r["flags"].sum()) == ref["n_discr"]
            assert np.array_equal(r["rk"], ref["keys"]) and np.array_equal(r["rc"], ref["counts"])
            assert np.array_equal(r["d0k"], ref["dumps"][0][0]) and np.array_equal(r["d0c"], ref["dumps"][0][1])
        else:
            assert len(r["keys"]) == 0 and len(r["rk"]) == 0 and len(r["d0k"]) == 0
