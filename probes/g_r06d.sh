# Round 6: stencil GPU tests of the product library, matcher variant timings,
# and a short bench of the product library with the large-batch drop-in legs.
# usage (on the box): bash probes/g_r06d.sh SET
set -e
S=${1:-r06d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_stencil.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > $O/stencil_tests.log 2>&1
TESTLIB=dva bash probes/g_r06a.sh $S base dvm dva dvah
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --extract-frames 0 \
  > $O/bench.log 2>&1
