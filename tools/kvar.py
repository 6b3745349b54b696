#!/usr/bin/env python3
"""Compare libhga tuning variants (tools/build_variants.sh) on the C2 count step, each in its own
process (HGA_LIB), after checking its result against the default build's row count / histogram."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import os, sys, json
sys.path[:0] = [%r, %r]
import bench, hga
ga, gb, ra, rb = bench.make_c2(0)
ctx = hga.Ctx(0); ctx.count_begin(19, 2); ctx.count_add(0, ra.seq); ctx.count_add(1, rb.seq)
def step():
    try:
        return bench.count_step(ctx)
    except hga.HgaError as e:   # timing-experiment variants may produce wrong data on purpose
        return str(e)[:60]
for _ in range(2): step()
ctx.profile(True); ctx.profile_reset()
import time; ctx.sync(); t0 = time.perf_counter()
for _ in range(10): n = step()
ctx.sync(); dt = (time.perf_counter() - t0) / 10
names = ("kc_init", "kc_bin1", "kc_layout", "kc_rebin", "kc_count", "kc_spec_hist", "kc_select", "radix_upsweep", "radix_downsweep", "bx_colscan", "bx_scatter", "radix_segsort")
try:
    hs = int(ctx.spec_hist(bench.THRESHOLDS)[:, 2].sum())
except hga.HgaError:
    hs = None
print(json.dumps({"ms": round(dt * 1e3, 3), "sel": n, "hist_sum": hs,
                  "k": {x: round(ctx.profile_get(x)[0] / 10, 4) for x in names}}))
''' % (ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd"))

for arg in sys.argv[1:]:   # path.so or path.so@ENV=V,ENV2=V
    so, _, envs = arg.partition("@")
    env = dict(os.environ, HGA_LIB=so)
    for kv in filter(None, envs.split(",")):
        k, _, v = kv.partition("=")
        env[k] = v
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
    line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-500:]
    print(os.path.basename(so) + ("@" + envs if envs else ""), line, flush=True)
