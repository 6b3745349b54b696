#!/usr/bin/env python3
"""C3 lookup timing of libhga variants (each in its own process): python tools/lkvar.py a.so b.so"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, json
sys.path[:0] = [%r, %r]
import bench, hga
ga, gb, ra, rb = bench.make_c2(0)
ctx = hga.Ctx(0); ctx.count_begin(19, 2); ctx.count_add(0, ra.seq); ctx.count_add(1, rb.seq); ctx.count_run(2)
sdk, _, _ = ctx.select(10, 25)
bases, offsets = bench.make_c3(ga, gb, 0)
c2 = hga.Ctx(0); c2.lookup_load(19, sdk); c2.lookup_set_reads(bases, offsets, 1); c2.lookup_run()
c2.profile(True); c2.profile_reset()
for _ in range(3): c2.lookup_run()
names = ("lk_pack", "lk_count", "lk_emit", "lk_post", "lk_sort", "lk_kci", "radix_segsort", "radix_upsweep", "radix_downsweep", "scan")
k = {n: round(c2.profile_get(n)[0] / 3, 4) for n in names}
c2.profile(False)
import time
c2.sync(); t0 = time.perf_counter()
for _ in range(10): c2.lookup_run()
c2.sync(); ms = (time.perf_counter() - t0) / 10 * 1e3
sz = c2.lookup_sizes()
print(json.dumps({"ms": round(ms, 3), "hits": int(sz.hits), "firsts": int(sz.firsts), "k": k}))
''' % (ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd"))
for arg in sys.argv[1:]:   # path.so or path.so@ENV=V,ENV2=V
    so, _, envs = arg.partition("@")
    env = dict(os.environ, HGA_LIB=so)
    for kv in filter(None, envs.split(",")):
        env[kv.partition("=")[0]] = kv.partition("=")[2]
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
    print(os.path.basename(so) + ("@" + envs if envs else ""), (out.stdout.strip().splitlines() or [out.stderr[-400:]])[-1],
          flush=True)
