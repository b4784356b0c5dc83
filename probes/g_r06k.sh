# Round 6: finalize-chain rowcheck chunk sizes (isolated matcher probe) and
# the F scoring kernel with two models per pass (SCM_VAR_FNM build): its
# verification GPU tests and a same-box bench A/B against the current build.
# usage (on the box): bash probes/g_r06k.sh SET
set -e
S=${1:-r06k}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
TESTLIB=rc64 bash probes/g_r06a.sh $S cur rc128 rc64
SCM_LIB=$R/probes/build/fnm/libscm.so timeout -k 10 500 python -u -m pytest tests/test_gpu_verify.py \
  tests/test_gpu_outcomes.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > $O/fnm_tests.log 2>&1
A="--steps 5 --warmup 2 --no-cpu-baseline --cpu-baseline-pairs 0 --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  SCM_LIB=$R/probes/build/cur/libscm.so timeout -k 10 300 python -u bench.py $A > $O/ab_cur_$i.log 2>&1
  SCM_LIB=$R/probes/build/fnm/libscm.so timeout -k 10 300 python -u bench.py $A > $O/ab_fnm_$i.log 2>&1
done
