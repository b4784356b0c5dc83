#!/bin/bash
# Diagnostics: libscm.so variants from edited copies of match_kernels.hip
# (one sed expression per variant), linked with the product's other objects:
# probes/build/<name>/libscm.so.
# usage: bash probes/build_match_sed.sh name:'s/kRcChunk = 256;/kRcChunk = 128;/' ...
set -e
cd "$(dirname "$0")/.."
make -C scanner_colmap_amd/csrc -s
O=scanner_colmap_amd/lib/obj
C=scanner_colmap_amd/csrc
for spec in "$@"; do
  name=${spec%%:*}; expr=${spec#*:}
  mkdir -p probes/build/$name
  sed "$expr" $C/match_kernels.hip > $C/_m_$name.hip
  cmp -s $C/match_kernels.hip $C/_m_$name.hip && { echo "variant $name: no change"; rm -f $C/_m_$name.hip; exit 1; }
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall \
    -c $C/_m_$name.hip -o probes/build/$name/match_kernels.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  rm -f $C/_m_$name.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o probes/build/$name/libscm.so \
    probes/build/$name/match_kernels.o $O/verify_kernels.o $O/sift_kernels.o $O/scm_runtime.o \
    $O/scm_codec.o $O/scm_sift.o
  echo "built probes/build/$name/libscm.so ($(sha256sum probes/build/$name/libscm.so | cut -c1-16))"
done
