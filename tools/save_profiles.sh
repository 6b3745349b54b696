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
# SQ / LDS counter passes (tools/gpu_pmc_sq.sh, tools/gpu_pmc_lds.sh), when present
[ -f gpurun_out/pmc_$TAG.json ] && cp gpurun_out/pmc_$TAG.json profiles/${TAG}_sq_pmc.json
ls -d gpurun_out/pmc_${TAG}_SQ_* >/dev/null 2>&1 && python3 tools/pmc_raw.py "gpurun_out/pmc_${TAG}_SQ_*" kc_bin1 kc_rebin kc_count_s kc_spec_hist kc_select rs_onesweep ss_segsort lk_scan hll_scan cn_wave > profiles/${TAG}_sq_lds_counters.txt
true
