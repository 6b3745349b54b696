#!/usr/bin/env python3
"""Compare libhga tuning variants (tools/build_variants.sh) on the C3 lookup, each in its own
process (HGA_LIB); prints ms, per-kernel ms and a checksum of the outputs."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import os, sys, json, time, hashlib
sys.path[:0] = [%r, %r]
import numpy as np, bench, hga
ga, gb, ra, rb = bench.make_c2(0)
ctx = hga.Ctx(0); ctx.count_begin(19, 2); ctx.count_add(0, ra.seq); ctx.count_add(1, rb.seq)
ctx.count_run(2); sdk, _, _ = ctx.select(10, 25)
bases, offsets = bench.make_c3(ga, gb, 0)
c2 = hga.Ctx(0); c2.lookup_load(19, sdk); c2.lookup_set_reads(bases, offsets, 1)
c2.lookup_run(); c2.profile(True); c2.profile_reset(); c2.sync(); t0 = time.perf_counter()
for _ in range(3): c2.lookup_run()
c2.sync(); dt = (time.perf_counter() - t0) / 3
r = c2.lookup_fetch(); h = hashlib.sha1()
for k in sorted(r): h.update(np.ascontiguousarray(r[k]).tobytes())
names = ("lk_count", "lk_emit", "lk_post", "lk_sort", "radix_upsweep", "radix_downsweep", "scan")
print(json.dumps({"ms": round(dt * 1e3, 3), "sha": h.hexdigest()[:12], "H": int(c2.lookup_sizes().hits), "k": {x: round(c2.profile_get(x)[0] / 3, 3) for x in names}}))
''' % (ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd"))

for so in sys.argv[1:]:
    env = dict(os.environ, HGA_LIB=so)
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
    line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-800:]
    print(os.path.basename(so), line, flush=True)
