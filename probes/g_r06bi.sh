# Round 6: Scanner op calls of 16 and 64 stencils under the system HIP runtime
# with every event of the library created without timing
# (probes/build/libscm_untimed.so) vs the product library, after a first
# plain process.
# usage (on the box): bash probes/g_r06bi.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_first.log 2>&1
for i in 1 2; do
  for v in untimed prod; do
    L=$R/scanner_colmap_amd/lib/libscm.so
    [ $v = untimed ] && L=$R/probes/build/libscm_untimed.so
    SCM_LIB=$L ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_${v}_$i.log 2>&1
    SCM_LIB=$L ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_${v}_$i.log 2>&1
  done
done
