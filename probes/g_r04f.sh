# Round 4: streamed passes (GPU tests of the pipeline, bench streamed vs one
# call per step, alternating), then the full -m gpu suite and smoke.
# usage (on the box): bash probes/g_r04f.sh SET
set -e
S=${1:-r04f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests_pipeline.log 2>&1
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --stencil-rows 0 --extract-frames 0 --no-isolated"
for i in 1 2; do
  timeout -k 10 300 python -u $B > $O/bench_stream_$i.log 2>&1
  timeout -k 10 300 python -u $B --no-stream > $O/bench_nostream_$i.log 2>&1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
