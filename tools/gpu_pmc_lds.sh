#!/bin/bash
# LDS-side PMC passes (one rocprofv3 run per counter group) over tools/kprof.py: bash tools/gpu_pmc_lds.sh <tag>
TAG=$1; shift
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for p in "SQ_LDS_ADDR_CONFLICT SQ_LDS_ATOMIC_RETURN SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INSTS_VALU_INT64 SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS" "SQ_INSTS_LDS_ATOMIC SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU"; do
  n=$(echo $p | cut -d" " -f1)
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $R/gpurun_out/pmc_${TAG}_$n -o run -- python3 $R/tools/kprof.py --reps 2 "$@" > $R/gpurun_out/pmc_${TAG}_$n.log 2>&1 || { echo "pmc $n failed"; tail -3 $R/gpurun_out/pmc_${TAG}_$n.log; exit 1; }
done
