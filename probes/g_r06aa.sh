# Round 6: the run's last batch with windows up to 64 rounds (SCM_VAR_LASTWIDE
# build, probes/build/lw) against the shipped library (probes/build/new):
# table-path GPU tests on lw, bench A/B alternating three times.
# usage (on the box): bash probes/g_r06aa.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
SCM_LIB=$R/probes/build/lw/libscm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py \
  tests/test_gpu_pipeline.py tests/test_gpu_verify.py tests/test_gpu_outcomes.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests_lw.log 2>&1
A="--steps 5 --warmup 2 --no-cpu-baseline --cpu-baseline-pairs 0 --stencil-rows 0 --extract-frames 0"
for i in 1 2 3; do
  for v in new lw; do
    SCM_LIB=$R/probes/build/$v/libscm.so timeout -k 10 300 python -u bench.py $A > $O/ab_${v}_$i.log 2>&1
  done
done
