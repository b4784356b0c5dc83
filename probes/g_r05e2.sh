# Round 5: small batches' verification enqueued before the counts reach the
# host (early enqueue): full GPU suite, batch-1 latency against
# SCM_EARLY_VERIFY=0 alternating, bench.
# usage (on the box): bash probes/g_r05e2.sh SET
set -e
S=${1:-r05e2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2 3; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_early_$i.log 2>&1
  SCM_EARLY_VERIFY=0 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_late_$i.log 2>&1
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline --extract-frames 0 > $O/bench.log 2>&1
