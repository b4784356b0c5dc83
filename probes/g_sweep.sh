# Diagnostics (GPU box): default bench under env settings, one line each.
# usage: bash probes/g_sweep.sh SET "ENV=V ..." ["ENV=V ..."]
set -e
S=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for cfg in "$@"; do
  echo "== $cfg" >> $O/sweep.log
  env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --stencil-rows 0 --cpu-baseline-pairs 0 2>&1 | grep '^{' >> $O/sweep.log
done
