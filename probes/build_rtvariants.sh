#!/bin/bash
# Builds libscm.so variants from edited copies of scm_runtime.cpp
# (diagnostics): probes/build/libscm_<name>.so, one sed expression per variant.
# usage: probes/build_rtvariants.sh name:'s/kOpCallBatches = 2;/kOpCallBatches = 3;/' ...
set -e
cd "$(dirname "$0")/.."
mkdir -p probes/build
make -C scanner_colmap_amd/csrc -s
O=scanner_colmap_amd/lib/obj
C=scanner_colmap_amd/csrc
for spec in "$@"; do
  name=${spec%%:*}; expr=${spec#*:}
  sed "$expr" $C/scm_runtime.cpp > $C/_r_$name.cpp
  cmp -s $C/scm_runtime.cpp $C/_r_$name.cpp && { echo "variant $name: no change"; exit 1; }
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall \
    -Wno-unused-result -x hip -c $C/_r_$name.cpp -o probes/build/rt_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  rm -f $C/_r_$name.cpp
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o probes/build/libscm_$name.so \
    $O/match_kernels.o $O/verify_kernels.o $O/sift_kernels.o probes/build/rt_$name.o \
    $O/scm_codec.o $O/scm_sift.o
done
