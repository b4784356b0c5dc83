# Round 5: GPU suite on the watermark index-vector fix, the bench, and the
# diagnostic's teeth (the fix reverted in a variant build: the scribble test
# must fail there).
# usage (on the box): bash probes/g_r05a.sh SET
set -e
S=${1:-r05a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
set +e
SCM_LIB=$R/probes/build/libscm_fsidx.so timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_stencil.py -k watermark_index_vector > $O/teeth.log 2>&1
echo "teeth rc $?" >> $O/teeth.log
exit 0
