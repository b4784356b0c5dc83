# Round 6: Scanner op calls of 16 and 64 stencils under the system HIP runtime
# with the stage events created without hipEventReleaseToDevice
# (probes/build/libscm_nortd.so) vs the product library, alternating.
# usage (on the box): bash probes/g_r06ax.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for i in 1 2 3; do
  for v in nortd prod; do
    L=$R/scanner_colmap_amd/lib/libscm.so
    [ $v = nortd ] && L=$R/probes/build/libscm_nortd.so
    SCM_LIB=$L ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_${v}_$i.log 2>&1
  done
done
for v in nortd prod; do
  L=$R/scanner_colmap_amd/lib/libscm.so
  [ $v = nortd ] && L=$R/probes/build/libscm_nortd.so
  SCM_LIB=$L ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_${v}.log 2>&1
  SCM_LIB=$L ROWS=64 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b1_${v}.log 2>&1
done
