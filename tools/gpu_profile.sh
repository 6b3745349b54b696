#!/bin/bash
# Round profile artifacts (run on the GPU box from the repo root):
#   1) rocprofv3 --kernel-trace --stats of the bench command itself  -> gpurun_out/stats_<tag>/
#   2) separate --pmc passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md §HBM: never combined
#      with other traces) over tools/kprof.py --lookup                   -> gpurun_out/hbm_<tag>_*/
#   3) per-kernel HBM bytes per launch                                  -> gpurun_out/pmc_<tag>/pmc_<kernel>.json
# usage: bash tools/gpu_profile.sh <tag> [bench args]
TAG=$1; shift
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/stats_$TAG -o run -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-scale "$@" > $R/gpurun_out/stats_$TAG.json 2> $R/gpurun_out/stats_$TAG.err \
    || { echo "stats run failed"; tail -5 $R/gpurun_out/stats_$TAG.err; exit 1; }
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $R/gpurun_out/hbm_${TAG}_$p -o run -- \
      python3 $R/tools/kprof.py --reps 2 --lookup --connections --hll > $R/gpurun_out/hbm_${TAG}_$p.log 2>&1 \
      || { echo "pmc $p failed"; tail -3 $R/gpurun_out/hbm_${TAG}_$p.log; exit 1; }
done
cd $R && python3 tools/pmc_summary.py gpurun_out/hbm_${TAG}_* --json gpurun_out/hbm_$TAG.json > gpurun_out/hbm_$TAG.txt \
  && python3 tools/make_pmc_json.py gpurun_out/hbm_$TAG.json gpurun_out/pmc_$TAG && cat gpurun_out/hbm_$TAG.txt
