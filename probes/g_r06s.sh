# Round 6: the product build with one descriptor upload per stage, the 2-D
# gather grid, the begin kernel's batched loads and the branch-free inlier
# compaction of the row serialisation: the whole GPU suite, per-call latency
# at batch 1 (HEAD build, cp = without the branch-free compaction, product),
# parallel LO chains for two windows (lo2), host step times (probes/build/ht),
# and bench A/B (HEAD vs product, with the
# drop-in legs).
# usage (on the box): bash probes/g_r06s.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
SCM_LIB=$R/probes/build/ht/libscm.so ROWS=24 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_ht.log 2>&1
bash probes/g_r06p.sh $S head cp lo2
A="--steps 5 --warmup 2 --no-cpu-baseline --cpu-baseline-pairs 0 --extract-frames 0"
SCM_LIB=$R/probes/build/head/libscm.so timeout -k 10 400 python -u bench.py $A > $O/ab_head_1.log 2>&1
timeout -k 10 400 python -u bench.py $A > $O/ab_new_1.log 2>&1
