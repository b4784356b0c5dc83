# Round 6: host step times (SCM_DIAG_HOST_TIMES build, probes/build/ht) and
# per-call stage times of Scanner op batches of 16 and 64 stencils.
# usage (on the box): bash probes/g_r06af.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for B in 16 64; do
  SCM_LIB=$R/probes/build/ht/libscm.so ROWS=$((B * 6)) B=$B timeout -k 10 300 python -u probes/stencil_probe.py > $O/stencil_ht_b$B.log 2>&1
done
