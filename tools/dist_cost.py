#!/usr/bin/env python3
"""One-GPU cost of the N>1 counting step's device work without the network: local
count (min 1), owner partition for `--owners` ranks, and the owner merge of as many pieces as this
rank sent (balanced owners receive about that many), then spec_hist + select.  Prints ms per phase."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import hga  # noqa: E402
import hga_dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--owners", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    ga, gb, ra, rb = bench.make_c2(0)
    ctx = hga.Ctx(0)
    ctx.count_begin(bench.K, 2)
    ctx.count_add(0, ra.seq)
    ctx.count_add(1, rb.seq)
    e = hga_dist.HgaEngine(ctx, bench.K, 2, "cuda:0")
    spl = hga_dist.owner_splitters(bench.K, a.owners)
    names = ("kc_pack", "kc_bin1", "kc_layout", "kc_rebin", "kc_count", "kx_partition", "kx_merge", "kx_piece_hist",
             "kx_pack_scatter", "kx_mb_hist", "kx_mb_scatter", "kx_mb_merge", "kx_mb_compact",
             "kc_spec_hist", "kc_select", "radix_upsweep", "radix_downsweep", "radix_segsort", "scan")
    t = {"count_local": 0.0, "partition": 0.0, "merge": 0.0, "hist+select": 0.0}
    for rep in range(a.reps + 1):
        if rep == 1:
            ctx.profile(True)
            ctx.profile_reset()
            t = {k: 0.0 for k in t}
        ctx.sync()
        t0 = time.perf_counter()
        rows = e.count_local()
        ctx.sync()
        t1 = time.perf_counter()
        cap = rows + rows // 64 + 1024
        buf = torch.empty(cap, dtype=torch.int64, device="cuda:0")
        per, total = e.partition_packed(spl, buf, cap)
        ctx.sync()
        t2 = time.perf_counter()
        e.merge_packed(buf, total, 2)
        ctx.sync()
        t3 = time.perf_counter()
        e.spec_hist(bench.THRESHOLDS)
        e.select_device(bench.LOWER, bench.UPPER)
        ctx.sync()
        t4 = time.perf_counter()
        for k, v in zip(t, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            t[k] += v * 1e3
    print("rows_local", rows, "pieces", total, "owners", a.owners)
    print({k: round(v / a.reps, 3) for k, v in t.items()})
    print({n: round(ctx.profile_get(n)[0] / a.reps, 4) for n in names if ctx.profile_get(n)[1]})


if __name__ == "__main__":
    main()
