#!/usr/bin/env python3
"""Counting at larger-than-C2 sizes on one GPU: a diploid pair of `--len` bp haplotypes at
`--cov`x ART-like 150 bp reads (2 files), k=19, count_run(2) + spec_hist + select_device.
Prints per-run ms, instances/s, buckets and the largest sub-range split (kc_count_s's table
overflow fallback), and checks the conservation identity (sum of counts + dropped = instances)
by the min-1 run.  e.g. --len 500000000 --cov 3.75 is one rank's shard of SURVEY.md's C4."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd")]
import hga  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--len", type=int, default=50_000_000)
    ap.add_argument("--cov", type=float, default=30.0)
    ap.add_argument("--div", type=float, default=0.005)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--k", type=str, default="19", help="comma-separated k values (SURVEY.md C5: 15,17,19,21)")
    a = ap.parse_args()
    t0 = time.time()
    ga = hga.gen_genome(a.len, 11)
    gb = hga.gen_haplotype(ga, a.div, 0, 12)
    n = int(a.cov * a.len / 150)
    ra = hga.gen_art(ga, n, 150, 13)
    rb = hga.gen_art(gb, n, 150, 14)
    print(f"generated {2 * n} reads, {len(ra.seq) + len(rb.seq)} bytes in {time.time() - t0:.1f}s", flush=True)
    ctx = hga.Ctx(0)
    for k in [int(x) for x in a.k.split(",")]:
        run_k(ctx, k, ra, rb, a.reps)
    ctx.close()


def run_k(ctx, k, ra, rb, reps):
    ctx.count_begin(k, 2)
    ctx.count_add(0, ra.seq)
    ctx.count_add(1, rb.seq)
    for rep in range(reps):
        ctx.profile(True)
        ctx.profile_reset()
        ctx.sync()
        t = time.perf_counter()
        ctx.count_run(2)
        ctx.spec_hist([70.0, 85.0, 90.0, 95.0, 99.0, 100.0, 100.01])
        sel = ctx.select_device(10, 25)
        ctx.sync()
        ms = (time.perf_counter() - t) * 1e3
        st = ctx.count_stats()
        names = ("kc_init", "kc_bin1", "kc_layout", "kc_rebin", "kc_split3", "kc_count", "kc_spec_hist", "kc_select",
                 "radix_upsweep", "radix_downsweep", "radix_segsort", "scan")
        ker = {nm: round(ctx.profile_get(nm)[0], 3) for nm in names if ctx.profile_get(nm)[1]}
        print(f"k={k} rep {rep}: {ms:.2f} ms, {st.instances / ms / 1e6:.1f} G k-mers/s, instances {st.instances}, "
              f"rows {st.distinct_rows}, buckets {st.buckets}, max_split {st.max_split}, selected {sel} {ker}",
              flush=True)
    ctx.count_run(1)
    st = ctx.count_stats()
    keys, cnts = ctx.rows()
    tot = int(cnts.astype("uint64").sum())
    print(f"k={k} min-1 rows {st.distinct_rows}, sum of counts {tot}, instances {st.instances}, identity "
          f"{'OK' if tot == st.instances else 'FAIL'}", flush=True)


if __name__ == "__main__":
    main()
