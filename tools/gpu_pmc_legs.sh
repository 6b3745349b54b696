#!/bin/bash
# PMC passes over one leg of kprof.py (each pass its own rocprofv3 run, counters per block
# within the limits of MI355X_MICROARCH.md).
# usage (on the box, repo root): bash tools/gpu_pmc_legs.sh <tag> <kprof args...>
TAG=$1; shift
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $R/gpurun_out/pmc_${TAG}_$i -o run -- \
      python3 $R/tools/kprof.py --reps 2 "$@" > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $R/gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_* --json gpurun_out/pmc_$TAG.json
