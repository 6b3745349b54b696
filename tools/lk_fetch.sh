#!/bin/bash
# lk_scan timing + FETCH_SIZE per libhga variant: bash tools/lk_fetch.sh <tag> lib1.so lib2.so ...
TAG=$1; shift
R=$PWD; mkdir -p gpurun_out
timeout -k 10 400 python3 tools/lkvar.py "$@" > gpurun_out/lkf_${TAG}.txt 2>&1 || { echo "lkvar failed"; tail -5 gpurun_out/lkf_${TAG}.txt; exit 1; }
cut -c1-300 gpurun_out/lkf_${TAG}.txt
export TMPDIR=/tmp
for so in "$@"; do
  n=$(basename $so .so)
  (cd /tmp && HGA_LIB=$so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/lkf_${TAG}_$n -o run -- python3 $R/tools/kprof.py --reps 2 --lookup > $R/gpurun_out/lkf_${TAG}_$n.log 2>&1) || { echo "pmc $n failed"; tail -3 gpurun_out/lkf_${TAG}_$n.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/lkf_${TAG}_$n 2>&1 | grep -i "kernel\|lk_scan" | cut -c1-60 | sed "s/^/$n /"
done
