# A/B of the 16x16x64 matcher (SCM_MATCH16=1) against the 32x32x32 one:
# matcher GPU tests under g16, then short benches alternating the two.
# usage (on the box): bash probes/g_m16.sh SET
set -e
S=${1:-m16}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 60 ./probes/build/mfma_shape > $O/mfma_shape.log 2>&1 || true
SCM_MATCH16=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_g16.log 2>&1
B="bench.py --steps 5 --warmup 2 --no-cpu-baseline --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  timeout -k 10 200 python -u $B > $O/bench_g8_$i.log 2>&1
  SCM_MATCH16=1 timeout -k 10 200 python -u $B > $O/bench_g16_$i.log 2>&1
done
