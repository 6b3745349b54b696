#!/usr/bin/env python3
"""get_all_connections(1) timing on C3 for libhga variants (each in its own process):
python tools/cnvar.py a.so b.so ...  Prints ms, per-kernel ms and a checksum of the output."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, json, time
import numpy as np
sys.path[:0] = [%r, %r]
import bench, hga
ga, gb, ra, rb = bench.make_c2(0)
ctx = hga.Ctx(0); ctx.count_begin(19, 2); ctx.count_add(0, ra.seq); ctx.count_add(1, rb.seq); ctx.count_run(2)
sdk, _, _ = ctx.select(10, 25)
bases, offsets = bench.make_c3(ga, gb, 0)
c2 = hga.Ctx(0); c2.lookup_load(19, sdk); c2.lookup_set_reads(bases, offsets, 1); c2.lookup_run()
n = c2.connections_run(min_kmers=1, min_score=1)
c2.profile(True); c2.profile_reset()
c2.sync(); t0 = time.perf_counter()
for _ in range(5): n = c2.connections_run(min_kmers=1, min_score=1)
c2.sync(); dt = (time.perf_counter() - t0) / 5
x, y = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
s, g = np.zeros(n, np.uint64), np.zeros(n, np.uint8)
hga.lib().hga_connections_fetch(c2._h, x.ctypes.data_as(hga._u32p), y.ctypes.data_as(hga._u32p),
                                s.ctypes.data_as(hga._u64p), g.ctypes.data_as(hga._u8p))
cs = int((x.astype(np.uint64) * 1000003 + y * 7 + s * 13).sum() %% (1 << 61))
names = ("cn_wave", "cn_local", "cn_global", "cn_sort", "radix_upsweep", "radix_downsweep", "scan")
print(json.dumps({"ms": round(dt * 1e3, 3), "n": int(n), "checksum": cs,
                  "k": {m: round(c2.profile_get(m)[0] / 5, 4) for m in names}}))
''' % (ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd"))
for arg in sys.argv[1:]:   # path.so or path.so@ENV=V,ENV2=V
    so, _, envs = arg.partition("@")
    env = dict(os.environ, HGA_LIB=so)
    for kv in filter(None, envs.split(",")):
        env[kv.partition("=")[0]] = kv.partition("=")[2]
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
    print(os.path.basename(so) + ("@" + envs if envs else ""), (out.stdout.strip().splitlines() or [out.stderr[-400:]])[-1],
          flush=True)
