#!/bin/bash
# Whole-bench comparison of libhga variants: bash tools/bvar.sh build_var/*.so  (one bench process each)
mkdir -p gpurun_out
for so in "$@"; do
  n=$(basename $so .so)
  HGA_LIB=$PWD/$so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-scale --no-ingest > gpurun_out/bv_$n.json 2> gpurun_out/bv_$n.err || { echo "$n failed"; tail -3 gpurun_out/bv_$n.err; exit 1; }
  python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.load(open(f"gpurun_out/bv_{n}.json"))
c = d["categorize"]
print(n, "count ms", d["ms_per_step"], {k: v for k, v in d["kernels_ms_per_step"].items()})
print(n, "  lookup ms", c["ms"], c["kernels_ms"])
print(n, "  conn ms", c["connections"]["ms"], c["connections"]["kernels_ms"])
PY
done
