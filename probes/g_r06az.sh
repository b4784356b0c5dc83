# Round 6: the table path's batch cap re-measured with the batch tables
# uploaded by kernel (SCM_BATCH_PAIRS: 8,192 default, 3 / 4 / 2 equal batches
# of the 18,810-pair step), alternating, two rounds.
# usage (on the box): bash probes/g_r06az.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0 --no-isolated"
for i in 1 2; do
  for BP in 8192 6272 4704 9408; do
    SCM_BATCH_PAIRS=$BP timeout -k 10 300 python -u bench.py $A > $O/bench_bp${BP}_$i.log 2>&1
  done
done
