#!/bin/bash
# GPU parity tests then a short bench; prints the headline numbers.  usage: bash tools/gpu_tb.sh <tag> [pytest -k expr]
TAG=$1; shift
mkdir -p gpurun_out
if [ -n "$1" ]; then K=(-k "$1"); else K=(); fi
timeout -k 10 600 python -m pytest tests -m gpu -x -q "${K[@]}" > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_$TAG.log | grep -v "^$" | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('ms/step', d['ms_per_step'], 'Gk/s', round(d['value']/1e9,2), 'split', d['config']['max_split'], 'frac', d['roofline']['frac'], d['roofline']['kernel']);print(d['kernels_ms_per_step']);print('lookup ms', d['categorize']['ms'], d['categorize']['kernels_ms'])"
