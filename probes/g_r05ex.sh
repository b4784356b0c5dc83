# Round 5: the exact kernel's batched qualification loads -- GPU suite on the
# new library, then the bench alternating with the shipped build
# (probes/build/libscm_base.so via SCM_LIB) on one box.
# usage (on the box): bash probes/g_r05ex.sh SET
set -e
S=${1:-r05ex}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so probes/build/libscm_base.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 900 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_outcomes.py tests/test_gpu_golden.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $A > $O/ab_new_$i.log 2>&1
  SCM_LIB=$R/probes/build/libscm_base.so timeout -k 10 300 python -u bench.py $A > $O/ab_base_$i.log 2>&1
done
