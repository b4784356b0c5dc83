# Round 6: the full GPU suite on the product library (new matcher schedule,
# switches removed), then a same-box bench A/B of the last batch on the
# small-batch kernels (SCM_VAR_LASTW=1, experiment) against the default.
# usage (on the box): bash probes/g_r06e.sh SET
set -e
S=${1:-r06e}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
A="--steps 5 --warmup 2 --no-cpu-baseline --cpu-baseline-pairs 0 --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/ab_base_$i.log 2>&1
  SCM_VAR_LASTW=1 timeout -k 10 300 python -u bench.py $A > $O/ab_lastw_$i.log 2>&1
done
