#!/bin/bash
# Build libhga variants with different compile-time tuning macros into /root/repo/build_var/<name>.so
# usage: tools/build_variants.sh name:"-DHGA_X=1 -DHGA_Y=2" ...
set -e -o pipefail
R=$(cd $(dirname $0)/.. && pwd); P=$R/hybrid-genome-assembler_amd
mkdir -p $R/build_var
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  d=$R/build_var/obj_$name; mkdir -p $d
  for f in sort count exchange comm lookup connect hll api; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/include -I$P/host $flags -c $P/csrc/$f.hip -o $d/$f.o &
  done
  wait || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $d/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o $R/build_var/$name.so
  rm -rf $d; echo "built $name ($flags)"
done
