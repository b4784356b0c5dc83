# Round 6: host-side step times of the SCM_DIAG_HOST_TIMES build (probes/build/
# ht, with collect / serialise split), and a small batch's window cap at 160 /
# 192 rounds (SCM_VAR_MAXW_SMALL builds) against the current sources (cp):
# per-call latency at batch 1, alternating on one box.
# usage (on the box): bash probes/g_r06r.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
SCM_LIB=$R/probes/build/ht/libscm.so ROWS=24 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_ht.log 2>&1
bash probes/g_r06p.sh $S cp w160 w192
