#!/bin/bash
# Builds a libscm.so variant from an edited copy of the whole source tree
# (diagnostics; for edits to headers the runtime shares):
# probes/build/libscm_<name>.so.
# usage: probes/build_treevariant.sh name FILE 'sed-expr' [FILE 'sed-expr' ...]
# (FILE relative to scanner_colmap_amd/csrc)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
T=/tmp/scm_var_$name
rm -rf $T && mkdir -p $T/scanner_colmap_amd $T/include
cp -r scanner_colmap_amd/csrc $T/scanner_colmap_amd/ && cp include/*.h $T/include/
while [ $# -ge 2 ]; do
  f=$T/scanner_colmap_amd/csrc/$1
  cp $f $f.orig && sed -i "$2" $f
  cmp -s $f $f.orig && { echo "variant $name: $1 unchanged"; exit 1; }
  rm $f.orig; shift 2
done
make -s -j8 -C $T/scanner_colmap_amd/csrc
cp $T/scanner_colmap_amd/lib/libscm.so probes/build/libscm_$name.so
rm -rf $T
