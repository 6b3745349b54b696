#!/bin/bash
# Kernel trace of tools/dist_step_times.py (one RCCL rank): bash tools/gpu_dsttrace.sh
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/dsttrace -o run -- python3 $R/tools/dist_step_times.py > $R/gpurun_out/dsttrace.log 2>&1
