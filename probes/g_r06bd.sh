# Round 6: Scanner op calls of 16 and 64 stencils under the system HIP runtime
# with the host-waited events (ev[3], ev[6]) created without timing
# (probes/build/libscm_notime36.so) vs the product library, after a first
# plain process.
# usage (on the box): bash probes/g_r06bd.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_first.log 2>&1
for i in 1 2; do
  for v in notime36 prod; do
    L=$R/scanner_colmap_amd/lib/libscm.so
    [ $v = notime36 ] && L=$R/probes/build/libscm_notime36.so
    SCM_LIB=$L ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_${v}_$i.log 2>&1
    SCM_LIB=$L ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_${v}_$i.log 2>&1
  done
done
