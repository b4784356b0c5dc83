# Round 6: finalize chain with the column merge in its own wide kernel
# (match_colmerge_g8_kernel) and the per-pair phases' loads batched (kFinU
# rows per thread), on top of the matcher's column split: GPU tests, per-call
# latency at batch 1 (HEAD build, column split only, both), and a kernel
# trace of the batch-1 calls.
# usage (on the box): bash probes/g_r06o.sh SET
set -e
S=${1:-r06o}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_stencil.py \
  tests/test_gpu_golden.py tests/test_gpu_outcomes.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  for lib in head split new; do
    L=$R/probes/build/$lib/libscm.so
    [ $lib = new ] && L=$R/scanner_colmap_amd/lib/libscm.so
    SCM_LIB=$L ROWS=24 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_${lib}_$i.log 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp
ROWS=12 B=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
