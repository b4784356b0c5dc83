# Round 4: small-batch windows of up to 128 rounds (product) vs 160 (F's
# 10,000 trials in two windows): batch-1 latency alternating; the product's
# per-stage profile with the worst pair of the final kernel.
# usage (on the box): bash probes/g_r04o.sh SET
set -e
S=${1:-r04o}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
V=$R/probes/build/libscm_win160.so
SCM_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_gpu_outcomes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_win160.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w128_$i.log 2>&1
  SCM_LIB=$V ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w160_$i.log 2>&1
done
ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile.log 2>&1
