#!/usr/bin/env python3
"""Shape of the connections workload on C3 (bench.py's generator): hits per read, pairs walked per
pivot, distinct candidates per pivot, list lengths.  Prints percentiles; used to size the
connection tiers (python tools/cnstats.py, on the GPU box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd")]
import bench  # noqa: E402
import hga  # noqa: E402


def pct(name, a):
    q = np.percentile(a, [0, 10, 50, 90, 99, 99.9, 100]) if len(a) else []
    print(f"{name:28s} n={len(a):9d} mean={np.mean(a) if len(a) else 0:10.1f} "
          + " ".join(f"{v:.0f}" for v in q), flush=True)


def main():
    ga, gb, ra, rb = bench.make_c2(0)
    ctx = hga.Ctx(0)
    ctx.count_begin(19, 2)
    ctx.count_add(0, ra.seq)
    ctx.count_add(1, rb.seq)
    ctx.count_run(2)
    sdk, _, _ = ctx.select(10, 25)
    bases, offsets = bench.make_c3(ga, gb, 0)
    c2 = hga.Ctx(0)
    c2.lookup_load(19, sdk)
    c2.lookup_set_reads(bases, offsets, 1)
    c2.lookup_run()
    f = c2.lookup_fetch()
    hp, kp, skid = f["hit_ptr"].astype(np.int64), f["kci_ptr"].astype(np.int64), f["sorted_kid"]
    hits = np.diff(hp)
    llen = np.diff(kp)
    pair_of_hit = llen[skid]
    pairs = np.add.reduceat(pair_of_hit, hp[:-1]) if len(pair_of_hit) else np.zeros(0)
    pairs[hits == 0] = 0
    rl = np.diff(offsets.astype(np.int64))
    x, y, s, g = c2.connections(min_kmers=1, min_score=1)
    distinct = np.bincount(x.astype(np.int64) - 1, minlength=len(hits))
    pct("read length", rl)
    pct("hits per read", hits)
    pct("kci list length (per kmer)", llen)
    pct("list length per hit", pair_of_hit)
    pct("pairs per pivot", pairs)
    pct("distinct cand per pivot", distinct)
    pct("score", s)
    for cap in (192, 384, 768, 1536):
        sel = distinct > cap
        print(f"distinct > {cap}: {sel.sum()} pivots, {pairs[sel].sum() / max(1, pairs.sum()):.3f} of pairs, "
              f"{hits[sel].sum() / max(1, hits.sum()):.3f} of hits", flush=True)
    # neighbouring hits of one read: how many list entries two consecutive KmerIDs of a read share
    print("hits", int(hits.sum()), "pairs", int(pairs.sum()), "connections", len(x), flush=True)


if __name__ == "__main__":
    main()
