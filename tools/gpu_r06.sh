#!/bin/bash
# One GPU call of round 6: tests, bench, rocprof stats, SQ/LDS counter passes, variant timings and the
# 2-rank rehearsal of bench --gpus N.  usage: bash tools/gpu_r06.sh <tag> [steps...]
#   steps (default all): test bench stats sq var gloo
TAG=$1; shift
STEPS=${*:-test bench stats sq var gloo}
R=$PWD; mkdir -p gpurun_out
export TMPDIR=/tmp
has() { [[ " $STEPS " == *" $1 "* ]]; }
set -o pipefail
if has test; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_$TAG.log
fi
if has ctest; then   # the counting tests only (count kernels, C2 / C4 sizes, export sort)
  timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_count_gpu.py \
    tests/test_export_sort_gpu.py tests/test_configs_gpu.py tests/test_scale_gpu.py > gpurun_out/ctest_$TAG.log 2>&1 \
    || { echo "ctest failed"; tail -30 gpurun_out/ctest_$TAG.log; exit 1; }
  tail -2 gpurun_out/ctest_$TAG.log
fi
if has bench; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('bench',d['ms_per_step'],d['value'],d['roofline']['frac'],d['categorize']['ms'],d['categorize']['connections']['ms'],d.get('scale_c4',{}).get('ms_per_step'))"
fi
if has stats; then
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/stats_$TAG -o run -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-scale --no-ingest > $R/gpurun_out/stats_$TAG.json 2> $R/gpurun_out/stats_$TAG.err) \
    || { echo "stats failed"; tail -5 gpurun_out/stats_$TAG.err; exit 1; }
  head -25 gpurun_out/stats_$TAG/*kernel_stats.csv | cut -c1-150
fi
if has sq; then
  for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_ADDR_CONFLICT SQ_LDS_ATOMIC_RETURN SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INSTS_VALU_INT64 SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS_ATOMIC" \
           "SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_INSTS_SMEM"; do
    n=$(echo $p | cut -d" " -f1)_$(echo $p | cut -d" " -f2)
    (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $R/gpurun_out/sq_${TAG}_$n -o run -- \
      python3 $R/tools/kprof.py --reps 2 --connections > $R/gpurun_out/sq_${TAG}_$n.log 2>&1) || { echo "pmc $n failed"; tail -3 gpurun_out/sq_${TAG}_$n.log; exit 1; }
  done
  python3 tools/pmc_raw.py "gpurun_out/sq_${TAG}_*" kc_bin1 kc_rebin kc_count_s lk_scan cn_wave > gpurun_out/sq_${TAG}.txt
  head -80 gpurun_out/sq_${TAG}.txt
fi
if has var; then
  L=$PWD/hybrid-genome-assembler_amd/lib/libhga.so; timeout -k 10 400 python3 tools/kvar.py $L $PWD/build_var/*.so $L $PWD/build_var/*.so > gpurun_out/var_$TAG.txt 2>&1 \
    || { echo "kvar failed"; tail -5 gpurun_out/var_$TAG.txt; exit 1; }
  cat gpurun_out/var_$TAG.txt | cut -c1-400
fi
if has gloo; then
  HGA_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/gloo2_$TAG.json \
    2> gpurun_out/gloo2_$TAG.err || { echo "gloo2 failed"; tail -8 gpurun_out/gloo2_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/gloo2_$TAG.json'));print('gloo2',d['n_gpus'],d['ms_per_step'],d.get('parity'),json.dumps(d.get('scale_c4'))[:600])"
fi
echo "gpu_r06 $TAG done"
