#!/bin/bash
# One GPU check on the box: selected parity tests, then the default bench line.
# usage (repo root on the box): bash tools/gpu_check.sh <tag> [test files...]
#   (no test files = the whole -m gpu suite)
TAG=$1; shift
mkdir -p gpurun_out
if [ $# -gt 0 ]; then T="$*"; else T="tests -m gpu"; fi
timeout -k 10 600 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python3 - "$TAG" <<'EOF'
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}.json"))
print("count: ms/step", d["ms_per_step"], "G k-mers/s", round(d["value"] / 1e9, 2), "roofline", d["roofline"]["kernel"],
      d["roofline"]["frac"])
print("kernels", d["kernels_ms_per_step"])
c = d.get("categorize", {})
print("lookup ms", c.get("ms"), c.get("kernels_ms"))
print("connections", {k: c.get("connections", {}).get(k) for k in ("ms", "kernels_ms")})
print("hll", c.get("hll_auto_k"))
print("ingest", d.get("ingest"))
EOF
