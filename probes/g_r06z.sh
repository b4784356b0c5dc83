# Round 6: the finalize chain's rowcheck / recheck with kFinLoop buckets /
# row groups per workgroup / wave on large batches (fewer workgroups beside
# the next batch's matcher; SCM_VAR_FINLOOP builds f1 / f8 / f32, the product
# f4): table-path GPU tests on f4, then bench A/B against the shipped build
# (the r06w library, probes/build/new).
# usage (on the box): bash probes/g_r06z.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fullsize.py tests/test_gpu_pipeline.py \
  tests/test_gpu_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
A="--steps 5 --warmup 2 --no-cpu-baseline --cpu-baseline-pairs 0 --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  for v in new f1 f4 f8; do
    SCM_LIB=$R/probes/build/$v/libscm.so timeout -k 10 300 python -u bench.py $A > $O/ab_${v}_$i.log 2>&1
  done
done
