# Diagnostics (GPU box): short bench runs (isolated stage times, pairs/s) of
# the libscm.so variants built by probes/build_vvariants.sh.
# usage: bash probes/g_vbench.sh SET v1 v2 ...
set -e
S=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for v in "$@"; do
  echo "== $v" >> $O/vbench.log
  SCM_LIB=probes/build/libscm_$v.so timeout -k 10 150 python -u bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --stencil-rows 0 --extract-frames 0 >> $O/vbench.log 2>&1
done
