# Round 5: skewed lane tables of the wave Shuffle (LDS banks): small-batch
# GPU tests, batch-1 latency (parallel LO off / first window), stage profile.
# usage (on the box): bash probes/g_r05e.sh SET
set -e
S=${1:-r05e}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_gpu_outcomes.py tests/test_scanner_op.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  SCM_PARALLEL_LO=0 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_off_$i.log 2>&1
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w1_$i.log 2>&1
done
SCM_PARALLEL_LO=0 ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile.log 2>&1
