# Round 6: op-call output elements copied on the worker pool (new) vs one
# thread (probes/build/libscm_prev.so): the bench's drop-in legs, alternating.
# usage (on the box): bash probes/g_r06bf.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
A="--steps 1 --warmup 0 --no-isolated --no-cpu-baseline --extract-frames 0 --stencil-batches 1:128,16:256,64:256,256:1024,512:1024"
for i in 1 2; do
  for v in new prev; do
    L=$R/scanner_colmap_amd/lib/libscm.so
    [ $v = prev ] && L=$R/probes/build/libscm_prev.so
    SCM_LIB=$L timeout -k 10 300 python -u bench.py $A > $O/bench_${v}_$i.log 2>&1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_scanner_op.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/stencil_tests.log 2>&1
