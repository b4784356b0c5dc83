# Round 4: small-batch windows of up to 128 rounds (H's 5,295 trials in two
# windows): batch-1 latency of this build (64) and the win128 variant,
# alternating; verification GPU tests on win128; a kernel trace of it.
# usage (on the box): bash probes/g_r04n.sh SET
set -e
S=${1:-r04n}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
V=$R/probes/build/libscm_win128.so
SCM_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_gpu_outcomes.py tests/test_gpu_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_win128.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w64_$i.log 2>&1
  SCM_LIB=$V ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w128_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
SCM_LIB=$V ROWS=12 B=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
