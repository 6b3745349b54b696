#!/usr/bin/env python3
"""C4 rank-shard count step (bench.py scale_leg) for libhga variants, each in its own process:
python tools/c4var.py a.so b.so ...   Prints ms/step, selected/discriminative and per-kernel ms."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, json
sys.path[:0] = [%r, %r]
import bench
r = bench.scale_leg(bench.Dist(1))
print(json.dumps({"ms": r["ms_per_step"], "sel": [r["selected"], r["discriminative"]], "k": r["kernels_ms_rank0"]}))
''' % (ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd"))
for arg in sys.argv[1:]:   # lib.so or lib.so:VAR=value,VAR2=value
    so, _, envs = arg.partition(":")
    env = dict(os.environ, HGA_LIB=so)
    for kv in filter(None, envs.split(",")):
        env[kv.split("=")[0]] = kv.split("=", 1)[1]
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=400)
    print(os.path.basename(arg), (out.stdout.strip().splitlines() or [out.stderr[-400:]])[-1], flush=True)
