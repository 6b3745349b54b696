#!/bin/bash
# Copy one GPU profiling call's summaries (tools/gpu_check.sh + tools/gpu_profile.sh <tag>) from
# gpurun_out/ into the tracked profiles/ directory: usage  bash tools/save_profiles.sh <tag>
set -e
TAG=$1
cp gpurun_out/bench_$TAG.json profiles/${TAG}_bench.json
cp gpurun_out/stats_$TAG.json profiles/${TAG}_bench_under_rocprof.json
cp gpurun_out/stats_$TAG/*kernel_stats.csv profiles/${TAG}_bench_kernel_stats.csv
cp gpurun_out/hbm_$TAG.json profiles/${TAG}_hbm_pmc.json
cp gpurun_out/hbm_$TAG.txt profiles/${TAG}_hbm_pmc.txt
cp gpurun_out/pmc_$TAG/pmc_*.json profiles/
tail -3 gpurun_out/pytest_$TAG.log > profiles/${TAG}_pytest_gpu.txt
