# Round 5: speculative watermark pass (verify_final_kernel phase 3) -- the
# full GPU suite, the watermark-index-vector teeth, batch-1 latency with the
# pass on / off (SCM_SPEC_WATERMARK=0), bench without the CPU baseline.
# usage (on the box): bash probes/g_r05j.sh SET
set -e
S=${1:-r05j}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_spec_$i.log 2>&1
  SCM_SPEC_WATERMARK=0 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_nospec_$i.log 2>&1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
