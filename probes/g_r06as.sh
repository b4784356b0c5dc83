# Round 6: Scanner op calls of 16 and 64 stencils under the system HIP runtime:
# the product library vs the host-times diagnostics build (probes/build/ht2),
# alternating.
# usage (on the box): bash probes/g_r06as.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for i in 1 2; do
  for v in prod ht2; do
    L=$R/scanner_colmap_amd/lib/libscm.so
    [ $v = ht2 ] && L=$R/probes/build/ht2/libscm.so
    SCM_LIB=$L ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_${v}_$i.log 2>&1
    SCM_LIB=$L ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_${v}_$i.log 2>&1
  done
done
