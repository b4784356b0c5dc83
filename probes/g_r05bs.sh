# Round 5: table path batch-cap sweep (SCM_BATCH_PAIRS) on the shipped
# library, alternating on one box.
# usage (on the box): bash probes/g_r05bs.sh SET
set -e
S=${1:-r05bs}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  for b in ${BPS:-8192 6270 9405 12544 4704}; do
    SCM_BATCH_PAIRS=$b timeout -k 10 300 python -u bench.py $A > $O/bp_${b}_$i.log 2>&1
  done
done
