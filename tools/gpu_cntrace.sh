cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/cntrace -o run -- python3 $R/tools/cnvar.py $R/hybrid-genome-assembler_amd/lib/libhga.so > $R/gpurun_out/cntrace.log 2>&1
