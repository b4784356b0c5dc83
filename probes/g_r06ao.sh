# Round 6: Scanner op calls cut into batches (run_rows kOpCallBatches /
# kOpCallEqualSplit; probes/build_rtvariants.sh): the bench's drop-in legs per
# library variant, alternating.
# usage (on the box): bash probes/g_r06ao.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
A="--steps 1 --warmup 0 --no-isolated --no-cpu-baseline --extract-frames 0 --stencil-batches 64:256,256:1024,512:1024"
for v in two one eq2 three two one; do
  L=$R/probes/build/libscm_$v.so
  [ $v = two ] && L=$R/scanner_colmap_amd/lib/libscm.so
  SCM_LIB=$L timeout -k 10 300 python -u bench.py $A > $O/bench_$v.$(date +%s).log 2>&1
done
