# Round 6: batch-1 call timeline (kernel trace) and the verification's
# per-phase cycle profile (SCM_PROFILE=1) of the product build.
# usage (on the box): bash probes/g_r06v.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile.log 2>&1
bash probes/g_stencil_trace.sh $S 1
