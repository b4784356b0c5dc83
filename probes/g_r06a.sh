# Round 6 (diagnostics): isolated matcher time of match_kernels.hip variants
# (probes/build_match_flags.sh), alternating, plus the matcher GPU tests on
# the variant with every change.  usage (on the box): bash probes/g_r06a.sh SET v1 v2 ...
set -e
S=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in "$@"; do
    IMAGES=${IMAGES:-120} REPS=3 TAG=$v timeout -k 10 120 python -u probes/matcher_probe.py \
      probes/build/$v/libscm.so >> $O/variants.log 2>&1
  done
done
if [ -n "$TESTLIB" ]; then
  SCM_LIB=$R/probes/build/$TESTLIB/libscm.so timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > $O/match_tests_$TESTLIB.log 2>&1
fi
