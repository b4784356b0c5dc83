# Round 6: Scanner op calls of 64 stencils unprofiled, with the process's HIP
# set-up varied: default, torch initialised first, device flags spin / yield /
# blocking sync (probes/stencil_probe.py PRE).
# usage (on the box): bash probes/g_r06an.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for P in none torch spin yield block; do
  PRE=$P ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_$P.log 2>&1
done
