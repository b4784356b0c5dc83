#!/bin/bash
# Diagnostics: libscm.so variants that differ only in match_kernels.hip,
# compiled with extra -D flags (experiment switches, removed from the source
# once a variant is kept or rejected) and linked with the product's other
# objects: probes/build/<name>/libscm.so for probes/matcher_probe.py and
# bench.py (SCM_LIB).
# usage: bash probes/build_match_flags.sh name:"-DFLAG ..." [name:"..."]
set -e
cd "$(dirname "$0")/.."
make -C scanner_colmap_amd/csrc -s
O=scanner_colmap_amd/lib/obj
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=probes/build/$name
  mkdir -p $out
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall $flags \
    -c scanner_colmap_amd/csrc/match_kernels.hip -o $out/match_kernels.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  out=probes/build/$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libscm.so $out/match_kernels.o \
    $O/verify_kernels.o $O/sift_kernels.o $O/scm_runtime.o $O/scm_codec.o $O/scm_sift.o
  echo "built $out/libscm.so ($(sha256sum $out/libscm.so | cut -c1-16))"
done
