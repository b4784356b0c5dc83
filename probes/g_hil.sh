# Round 4: stage-interleaved H split pass (two point pairs x kScoreHm models per
# step) vs the previous one-pair form: verification GPU tests on the new build,
# then alternating benches of both builds with the isolated leg.
# usage (on the box): bash probes/g_hil.sh SET
set -e
S=${1:-hil}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_outcomes.py tests/test_gpu_golden.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests_verify.log 2>&1
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --extract-frames 0"
for i in 1 2; do
  SCM_LIB=$R/probes/build/libscm_base.so timeout -k 10 300 python -u $B > $O/bench_base_$i.log 2>&1
  SCM_LIB=$R/probes/build/libscm_il.so timeout -k 10 300 python -u $B > $O/bench_il_$i.log 2>&1
done
