# Round 6: the small-batch threshold (kWaveShufflePairs, SCM_VAR_SMALLPAIRS
# builds t512 / t1024 / t2048) against the shipped 256 (new): drop-in legs at
# op batch 8-64 (152-1,216 pairs per call), alternating.
# usage (on the box): bash probes/g_r06ad.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
A="--steps 1 --warmup 1 --no-cpu-baseline --cpu-baseline-pairs 0 --extract-frames 0 --no-isolated"
for i in 1 2; do
  for v in new t512 t1024 t2048; do
    L=$R/probes/build/$v/libscm.so
    [ $v = new ] && L=$R/scanner_colmap_amd/lib/libscm.so
    SCM_LIB=$L timeout -k 10 400 python -u bench.py $A --stencil-batches 8:128,16:256,32:256,64:256 > $O/legs_${v}_$i.log 2>&1
  done
done
