#!/bin/bash
# Diagnostics: libscm.so variants that differ only in verify_kernels.hip,
# compiled with extra -D flags (experiment switches, removed from the source
# once a variant is kept or rejected): probes/build/<name>/libscm.so.
# usage: bash probes/build_verify_flags.sh name:"-DFLAG ..." [name:"..."]
set -e
cd "$(dirname "$0")/.."
make -C scanner_colmap_amd/csrc -s
O=scanner_colmap_amd/lib/obj
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p probes/build/$name
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall $flags \
    -c scanner_colmap_amd/csrc/verify_kernels.hip -o probes/build/$name/verify_kernels.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o probes/build/$name/libscm.so \
    $O/match_kernels.o probes/build/$name/verify_kernels.o $O/sift_kernels.o $O/scm_runtime.o \
    $O/scm_codec.o $O/scm_sift.o
  echo "built probes/build/$name/libscm.so ($(sha256sum probes/build/$name/libscm.so | cut -c1-16))"
done
