#!/usr/bin/env python3
"""HLL sweep timing (k = 11..31) of libhga variants, each in its own process: python tools/hllvar.py a.so b.so"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, time, json
sys.path[:0] = [%r, %r]
import bench, hga
ga, gb, ra, rb = bench.make_c2(0)
bases, offsets = bench.make_c3(ga, gb, 0)
ctx = hga.Ctx(0); ctx.lookup_set_reads(bases, offsets, 1)
ks = list(range(11, 33, 2))
regs = {kk: ctx.hll_registers(kk).tobytes().hex()[:16] for kk in ks}
ctx.profile(True); ctx.profile_reset()
for kk in ks: ctx.hll_registers(kk)
print(json.dumps({"hll_scan_ms_per_k": round(ctx.profile_get("hll_scan")[0] / len(ks), 4), "regs19": regs[19]}))
''' % (ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd"))
for so in sys.argv[1:]:
    out = subprocess.run([sys.executable, "-c", CODE], env=dict(os.environ, HGA_LIB=so), capture_output=True,
                         text=True, timeout=300)
    print(os.path.basename(so), (out.stdout.strip().splitlines() or [out.stderr[-400:]])[-1], flush=True)
