# Round 4: the small-batch final kernel (configuration + watermark RANSAC)
# with eight waves per pair instead of four: small-batch GPU tests on the
# variant, batch-1 latency alternating with this build, its stage profile.
# usage (on the box): bash probes/g_r04r.sh SET
set -e
S=${1:-r04r}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
V=$R/probes/build/libscm_fin8.so
SCM_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_gpu_outcomes.py tests/test_gpu_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_fin8.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_fin4_$i.log 2>&1
  SCM_LIB=$V ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_fin8_$i.log 2>&1
done
SCM_LIB=$V ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile_fin8.log 2>&1
