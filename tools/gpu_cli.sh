#!/bin/bash
# CLI parity tests + the bench's CLI legs (categorization pipeline, jf_occurrences) on the box.
# usage: bash tools/gpu_cli.sh <tag>
TAG=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_cli_gpu.py \
    tests/test_host.py > gpurun_out/pytest_cli_$TAG.log 2>&1 || { tail -20 gpurun_out/pytest_cli_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_cli_$TAG.log
timeout -k 10 300 python bench.py --no-scale > gpurun_out/bench_cli_$TAG.json 2> gpurun_out/bench_cli_$TAG.err \
    || { tail -5 gpurun_out/bench_cli_$TAG.err; exit 1; }
python3 - "$TAG" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/bench_cli_{sys.argv[1]}.json"))
p = d["categorize"]["pipeline"]; t = d["categorize"].get("pipeline_tails", {})
print("categorization wall", p["wall_s"], p["phases_ms"])
print("tails wall", t.get("wall_s"))
print("jf", d["ingest"]["cli_jf_occurrences"]["wall_s"])
PY
