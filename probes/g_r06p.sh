# Round 6: a small batch's second window sizes (SCM_VAR_W1H / SCM_VAR_W1F
# builds, probes/build_verify_flags.sh): per-call latency at batch 1 against
# the product build, alternating on one box.
# usage (on the box): bash probes/g_r06p.sh SET VARIANT...
set -e
S=$1
shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for i in 1 2; do
  for lib in new "$@"; do
    L=$R/probes/build/$lib/libscm.so
    [ $lib = new ] && L=$R/scanner_colmap_amd/lib/libscm.so
    SCM_LIB=$L ROWS=24 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_${lib}_$i.log 2>&1
  done
done
