#!/bin/bash
# Diagnostics: build libscm.so variants of the matcher (compile-time switches)
# into probes/build/<name>/libscm.so for probes/matcher_probe.py.
# usage: bash probes/build_match_variants.sh name:"-DFLAG ..." [name:"..."]
set -e
cd "$(dirname "$0")/../scanner_colmap_amd/csrc"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=../../probes/build/$name
  mkdir -p $out/obj
  for f in match_kernels verify_kernels sift_kernels; do
    /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off --offload-arch=gfx950 $flags -c $f.hip -o $out/obj/$f.o &
  done
  for f in scm_runtime scm_codec scm_sift; do
    /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off --offload-arch=gfx950 $flags -x hip -c $f.cpp -o $out/obj/$f.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libscm.so $out/obj/*.o
  echo built $out/libscm.so
done
