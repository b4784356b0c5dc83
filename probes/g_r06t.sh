# Round 6: the table path after the small-batch changes (matcher tile ranges,
# colmerge kernel, worker pool, serialisation): isolated matcher time HEAD vs
# product (g_r06a.sh), and bench A/B alternating three times.
# usage (on the box): bash probes/g_r06t.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
bash probes/g_r06a.sh $S head new
A="--steps 5 --warmup 2 --no-cpu-baseline --cpu-baseline-pairs 0 --stencil-rows 0 --extract-frames 0"
for i in 1 2 3; do
  SCM_LIB=$R/probes/build/head/libscm.so timeout -k 10 300 python -u bench.py $A > $O/ab_head_$i.log 2>&1
  timeout -k 10 300 python -u bench.py $A > $O/ab_new_$i.log 2>&1
done
