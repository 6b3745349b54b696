#!/usr/bin/env python3
"""Kernel-profiling driver: builds the C2 workload (bench.py's generator) and runs only the
device counting pipeline (and optionally the C3 lookup) a few times, so rocprofv3 --pmc passes
see the same kernels bench.py times without the CPU baseline or generation noise.

    rocprofv3 --pmc SQ_WAVES ... -- python3 tools/kprof.py --reps 3 [--lookup]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd")]
import bench  # noqa: E402
import hga  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lookup", action="store_true")
    ap.add_argument("--connections", action="store_true", help="also get_all_connections (implies --lookup)")
    ap.add_argument("--hll", action="store_true", help="also hll_registers k=19 (implies --lookup)")
    a = ap.parse_args()
    ga, gb, ra, rb = bench.make_c2(0)
    ctx = hga.Ctx(0)
    ctx.count_begin(bench.K, 2)
    ctx.count_add(0, ra.seq)
    ctx.count_add(1, rb.seq)
    for _ in range(a.reps):
        bench.count_step(ctx)
    st = ctx.count_stats()
    print(f"instances={st.instances} rows={st.distinct_rows} buckets={st.buckets} max_split={st.max_split}")
    if a.lookup or a.connections or a.hll:
        bases, offsets = bench.make_c3(ga, gb, 0)
        sdk, _, _ = ctx.select(bench.LOWER, bench.UPPER)
        ctx2 = hga.Ctx(0)
        ctx2.lookup_load(bench.K, sdk)
        ctx2.lookup_set_reads(bases, offsets, 1)
        for _ in range(a.reps):
            ctx2.lookup_run()
        print(f"hits={ctx2.lookup_sizes().hits}")
        for _ in range(a.reps if a.connections else 0):
            ctx2.connections_run(min_score=1)
        for _ in range(a.reps if a.hll else 0):
            ctx2.hll_registers(19)
        ctx2.close()
    ctx.close()


if __name__ == "__main__":
    main()
