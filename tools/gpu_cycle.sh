#!/bin/bash
# One GPU iteration: parity tests, short bench, PMC passes of the counting kernels.
# usage (on the box): bash tools/gpu_cycle.sh <tag> [pytest-args...]
TAG=$1; shift
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q "$@" > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('ms/step', d['ms_per_step'], 'Gk/s', round(d['value']/1e9,2), 'split', d['config']['max_split']);print(d['kernels_ms_per_step']);print('lookup ms', d['categorize']['ms'], d['categorize']['kernels_ms'])"
cd /tmp && export TMPDIR=/tmp
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU"; do
  n=$(echo $p | cut -d" " -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $R/gpurun_out/pmc_${TAG}_$n -o run -- python3 $R/tools/kprof.py --reps 2 > $R/gpurun_out/pmc_${TAG}_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
done
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_* --json gpurun_out/pmc_${TAG}.json
