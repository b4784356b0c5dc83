# Round 6: the 4-waves-per-SIMD model probe, matcher variant timings, and the
# stencil GPU tests of the product library (the new forced-order and
# parallel-LO cases).  usage (on the box): bash probes/g_r06c.sh SET
set -e
S=${1:-r06c}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 120 ./probes/build/mfma_model4 > $O/model4.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_stencil.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > $O/stencil_tests.log 2>&1
TESTLIB=dva bash probes/g_r06a.sh $S base dvm dva dvah base dvm dva dvah
