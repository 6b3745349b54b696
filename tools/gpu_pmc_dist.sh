#!/bin/bash
# SQ / LDS counter passes over tools/dist_step_times.py (one RCCL rank: owner partition + merge kernels).  usage: bash tools/gpu_pmc_dist.sh <tag>
TAG=$1; shift
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  n=$(echo $p | cut -d" " -f1)
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $R/gpurun_out/pmc_${TAG}_$n -o run -- python3 $R/tools/dist_step_times.py > $R/gpurun_out/pmc_${TAG}_$n.log 2>&1 || { echo "pmc $n failed"; tail -3 $R/gpurun_out/pmc_${TAG}_$n.log; exit 1; }
done
cd $R && python3 tools/pmc_raw.py "gpurun_out/pmc_${TAG}_*" kx_piece_hist kx_pack_scatter kx_mb_hist kx_mb_scatter kx_mb_merge kx_mb_compact
