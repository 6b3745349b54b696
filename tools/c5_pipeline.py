#!/usr/bin/env python3
"""BASELINE.json configs[4] ("C5"): the full pipeline for k in {15, 17, 19, 21} — k-mer counting and
SDK export (jf_occurrences), SDK lookup (categorization's construct_indices) and the shared-k-mer read
graph (get_all_connections) — on a human-chr1-scale synthetic diploid, one rank per GPU.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/c5_pipeline.py
    python tools/c5_pipeline.py --scale 0.01          # one rank, a 1 % sized genome
    HGA_BENCH_BACKEND=gloo torchrun ... --check       # ranks sharing one GPU, checked against the oracle

Every step goes through the C ABI (include/hga.h) with the library's own communicator (RCCL over
xGMI for backend nccl, the host transport hook otherwise; hga_dist.attach):
  count    each rank: its share of the ART-like 30x reads of both haplotypes; hga_count_run(1) +
           hga_count_exchange(2); the global histogram (hga_count_spec_hist) and
           export at [lower, upper] (hga_count_select_ex: the whole export on every rank);
  lookup   each rank: its contiguous ReadID range of the Nanosim-like long reads against the export
           (hga_lookup_run), hga_lookup_gather -> the whole index on every rank;
  graph    each rank connects its own reads (hga_connections_run, min_score 1) over the whole index,
           hga_connections_gather joins them (get_all_connections, ReadClusteringEngine.cpp:335-339).
Timed per k (barrier + device sync on both sides; an untimed pass of the first k runs before, so
first-use buffer allocations are not in any stage): the uploads of the short reads (hga_count_add) and
of the SDK table + long reads (hga_lookup_load / hga_lookup_set_reads) separately from the three device
stages count (run, exchange, histogram, export), lookup (run + gather) and graph.
Synthetic data (no simulators offline): genome i.i.d. ACGT, haplotype B with d = 0.001 substitutions;
reads from host/gen.cpp's ART-like / Nanosim-like generators, each rank drawing its
own share with its own seeds.  Rank 0 prints one JSON line with per-k stage times (max over ranks).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd")]
import hga  # noqa: E402

CHR1 = 248_956_422
THRESHOLDS = [70.0, 85.0, 90.0, 95.0, 99.0, 100.0, 100.01]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def shares(n, world):
    return [(n * r // world, n * (r + 1) // world) for r in range(world)]


def make_data(L, d, art_cov, lr_cov, rank, world):
    """This rank's ART-like short-read shards (per haplotype) and long-read shard (+ its first ReadID)."""
    ga = hga.gen_genome(L, 51)
    gb = hga.gen_haplotype(ga, d, 0, 52)
    n_art = int(art_cov * L / 150)
    a0, a1 = shares(n_art, world)[rank]
    art = [hga.gen_art(g, a1 - a0, 150, 1000 + 4 * rank + h) for h, g in enumerate((ga, gb))]
    n_lr = round(L / 7777 * lr_cov)
    lr, first = [], 1
    for h, g in enumerate((ga, gb)):
        b0, b1 = shares(n_lr, world)[rank]
        lr.append(hga.gen_nanosim(g, b1 - b0, 3000 + 4 * rank + h))
    # ReadIDs: haplotype A's long reads of every rank, then B's (reader order, SequenceRecordIterator
    # IDs from 1); this rank holds [b0, b1) of A and [b0, b1) of B -> two ranges.  To keep one
    # contiguous ReadID range per rank the rank's A and B reads are numbered together.
    counts = [shares(n_lr, world)[r][1] - shares(n_lr, world)[r][0] for r in range(world)]
    first = 1 + 2 * sum(counts[:rank])
    bases = lr[0].bases + lr[1].bases
    offsets = np.concatenate([lr[0].offsets, lr[1].offsets[1:] + lr[0].offsets[-1]]).astype(np.uint64)
    return ga, gb, art, bases, offsets, first


def run(rank, world, args, group_ready=False):
    if world > 1 and not group_ready:
        import torch
        import torch.distributed as dist
        backend = os.environ.get("HGA_BENCH_BACKEND", "nccl")
        local = int(os.environ.get("LOCAL_RANK", rank))
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    dev = int(os.environ.get("LOCAL_RANK", rank)) if os.environ.get("HGA_BENCH_BACKEND", "nccl") == "nccl" else 0
    if world > 1:
        import torch.distributed as dist
        barrier = dist.barrier
    else:
        def barrier():
            return None
    L = int(CHR1 * args.scale)
    t = time.perf_counter()
    ga, gb, art, lr_bases, lr_offsets, first_id = make_data(L, args.div, args.art_cov, args.lr_cov, rank, world)
    log(f"[rank {rank}] data in {time.perf_counter() - t:.1f}s: {sum(r.n for r in art)} short reads, "
        f"{len(lr_offsets) - 1} long reads from ReadID {first_id}")
    ctx = hga.Ctx(dev)
    if world > 1:
        import hga_dist
        hga_dist.attach(ctx)
    out = {"workload": f"C5: 2 x {L} bp synthetic diploid (d={args.div}), ART-like {args.art_cov}x 150 bp + "
                       f"Nanosim-like {args.lr_cov}x long reads; k in {args.ks}",
           "ranks": world, "per_k": {}}
    checks = {}

    def timed(fn):
        barrier()
        ctx.sync()
        t0 = time.perf_counter()
        r = fn()
        ctx.sync()
        barrier()
        return r, time.perf_counter() - t0

    for it, k in enumerate(([args.ks[0]] if args.warmup else []) + list(args.ks)):
        warm = args.warmup and it == 0   # untimed first pass: the device buffers' first allocations

        def upload_short():
            ctx.count_begin(k, 2)
            for f in range(2):
                ctx.count_add(f, art[f].seq)
        _, t_up_short = timed(upload_short)

        def count():
            if world > 1:
                ctx.count_run(1)
                ctx.count_exchange(2)
            else:
                ctx.count_run(2)
            hist = ctx.spec_hist(THRESHOLDS)
            sel, flags, nd = ctx.select(args.lower, args.upper)
            return hist, sel, nd
        (hist, sdk, nd), t_count = timed(count)
        st = ctx.count_stats()

        def upload_long():
            ctx.lookup_load(k, sdk)
            ctx.lookup_set_reads(lr_bases, lr_offsets, first_id)
        _, t_up_long = timed(upload_long)

        def lookup():
            ctx.lookup_run()
            if world > 1:
                ctx.lookup_gather()
            return ctx.lookup_sizes()
        sz, t_lookup = timed(lookup)

        def graph():
            n_own = len(lr_offsets) - 1
            piv = np.arange(first_id, first_id + n_own, dtype=np.uint32)
            n = ctx.connections_run(pivots=piv, min_kmers=1, min_score=1)
            return ctx.connections_gather() if world > 1 else n
        n_conn, t_graph = timed(graph)
        if warm:
            log(f"[rank {rank}] warm-up pass (k={k}) done")
            continue
        out["per_k"][k] = {"instances": int(st.instances), "distinct_rows": int(st.distinct_rows),
                           "exported": int(len(sdk)), "discriminative": int(nd),
                           "upload_short_reads_s": round(t_up_short, 4),
                           "count_s": round(t_count, 4), "k_mers_per_s": round(st.instances / t_count, 1),
                           "long_reads": int(sz.n_reads), "windows": int(sz.windows), "hits": int(sz.hits),
                           "upload_long_reads_and_sdk_s": round(t_up_long, 4),
                           "lookup_s": round(t_lookup, 4), "windows_per_s": round(sz.windows / t_lookup, 1),
                           "connections": int(n_conn), "graph_s": round(t_graph, 4),
                           "pipeline_device_s": round(t_count + t_lookup + t_graph, 4)}
        if args.check:
            checks[k] = {"hist": hist, "sdk": sdk, "nd": nd, "idx": ctx.lookup_fetch(), "conn": _fetch_conn(ctx, n_conn)}
        log(f"[rank {rank}] k={k}: {out['per_k'][k]}")
    ctx.close()
    if args.check and rank == 0:
        verify(args, world, checks, own=(ga, gb, art, lr_bases, lr_offsets, first_id) if world == 1 else None)
        out["checked_against_oracle"] = True
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1 and not group_ready:
        import torch.distributed as dist
        dist.destroy_process_group()
    return out


def _fetch_conn(ctx, n):
    x, y = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    s, g = np.zeros(n, np.uint64), np.zeros(n, np.uint8)
    hga.lib().hga_connections_fetch(ctx._h, x.ctypes.data_as(hga._u32p), y.ctypes.data_as(hga._u32p),
                                    s.ctypes.data_as(hga._u64p), g.ctypes.data_as(hga._u8p))
    return x, y, s


def verify(args, world, checks, own=None):
    """Rank 0 regenerates every rank's shards (same seeds; at one rank its own data is reused) and
    runs the oracle over all of them."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    L = int(CHR1 * args.scale)
    shards = [own] if own is not None else \
        [make_data(L, args.div, args.art_cov, args.lr_cov, r, world) for r in range(world)]
    streams = [b"\n".join(s[2][f].seq for s in shards) for f in range(2)]
    bases = b"".join(s[3] for s in shards)
    offs = [np.zeros(1, np.uint64)]
    base = 0
    for s in shards:
        offs.append(s[4][1:] + np.uint64(base))
        base += int(s[4][-1])
    offsets = np.concatenate(offs).astype(np.uint64)
    del shards
    th = args.check_threads
    for k, c in checks.items():
        t0 = time.perf_counter()
        if th > 1:   # the multi-threaded restatements (each checked against the plain one in tests/)
            o = oracle.count_pipeline_mt(streams, k, args.lower, args.upper, th)
        else:
            o = oracle.count_pipeline(streams, k, args.lower, args.upper)
        assert np.array_equal(c["hist"], o["hist"]), f"k={k}: histogram"
        assert np.array_equal(c["sdk"], o["selected"]) and c["nd"] == o["n_discr"], f"k={k}: export"
        sel = o["selected"]
        del o
        idx = oracle.construct_indices(bases, offsets, k, sel, 1, threads=th if th > 1 else 0)
        for name in idx:
            assert np.array_equal(c["idx"][name], idx[name]), f"k={k}: lookup {name}"
        if th > 1:
            x, y, s = oracle.connections_mt(idx, th, min_score=1)
        else:
            x, y, s, _ = oracle.connections(idx, min_score=1)
        assert np.array_equal(c["conn"][0], x) and np.array_equal(c["conn"][1], y) and \
            np.array_equal(c["conn"][2], s), f"k={k}: connections"
        log(f"k={k}: export ({len(sel)}), index ({len(idx['hit_kid'])} hits) and read graph ({len(x)} "
            f"connections) equal the oracle [{time.perf_counter() - t0:.1f}s]")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0, help="genome length as a fraction of human chr1")
    ap.add_argument("--ks", type=lambda s: [int(x) for x in s.split(",")], default=[15, 17, 19, 21])
    ap.add_argument("--div", type=float, default=0.001)
    ap.add_argument("--art-cov", type=float, default=30.0)
    ap.add_argument("--lr-cov", type=float, default=75.0)
    ap.add_argument("--lower", type=int, default=10)
    ap.add_argument("--upper", type=int, default=25)
    ap.add_argument("--check", action="store_true", help="rank 0 checks every stage against the oracle")
    ap.add_argument("--check-threads", type=int, default=1,
                    help="oracle threads for --check (> 1: the multi-threaded restatements)")
    ap.add_argument("--warmup", type=int, default=1, help="1: an untimed pass of the first k first (allocations)")
    return ap.parse_args(argv)


if __name__ == "__main__":
    a = parse()
    run(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), a)
