# A/B of two library builds on one box (diagnostics): bench.py table path
# with the default build and with $1 (an SCM_LIB path), alternating.
# usage: bash probes/g_ab.sh SET LIB [extra bench args]
set -e
S=$1
LIB=$2
shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/new_$i.log 2>&1
  SCM_LIB=$R/$LIB timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/old_$i.log 2>&1
done
