# Round 6: the finalize chain's rowcheck staging with every load in flight:
# matcher / full-size / pipeline GPU tests, then a bench with parity (the
# isolated finalize time).  usage (on the box): bash probes/g_r06i.sh SET
set -e
S=${1:-r06i}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fullsize.py \
  tests/test_gpu_pipeline.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --stencil-rows 0 \
  --extract-frames 0 > $O/bench.log 2>&1
