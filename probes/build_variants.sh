#!/bin/bash
# Builds libscm.so variants of the matcher (diagnostics): probes/build/libscm_<name>.so
# usage: probes/build_variants.sh name:"-DFOO=1 -DBAR=0" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p probes/build
make -C scanner_colmap_amd/csrc -s
O=scanner_colmap_amd/lib/obj
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off --offload-arch=gfx950 $defs \
    -c scanner_colmap_amd/csrc/match_kernels.hip -o probes/build/match_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o probes/build/libscm_$name.so \
    probes/build/match_$name.o $O/verify_kernels.o $O/sift_kernels.o $O/scm_runtime.o \
    $O/scm_codec.o $O/scm_sift.o
done
