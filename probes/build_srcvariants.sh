#!/bin/bash
# Builds libscm.so variants from edited copies of verify_kernels.hip
# (diagnostics): probes/build/libscm_<name>.so, one sed expression per variant.
# usage: probes/build_srcvariants.sh name:'s/kLoU = 4;/kLoU = 8;/' ...
set -e
cd "$(dirname "$0")/.."
mkdir -p probes/build
make -C scanner_colmap_amd/csrc -s
O=scanner_colmap_amd/lib/obj
C=scanner_colmap_amd/csrc
for spec in "$@"; do
  name=${spec%%:*}; expr=${spec#*:}
  sed "$expr" $C/verify_kernels.hip > $C/_v_$name.hip
  cmp -s $C/verify_kernels.hip $C/_v_$name.hip && { echo "variant $name: no change"; exit 1; }
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off --offload-arch=gfx950 \
    -c $C/_v_$name.hip -o probes/build/verify_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  rm -f $C/_v_$name.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o probes/build/libscm_$name.so \
    $O/match_kernels.o probes/build/verify_$name.o $O/sift_kernels.o $O/scm_runtime.o \
    $O/scm_codec.o $O/scm_sift.o
done
