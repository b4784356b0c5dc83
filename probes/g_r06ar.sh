# Round 6: host step times + GPU stage times from the call's start
# (SCM_DIAG_HOST_TIMES build probes/build/ht2) of Scanner op calls of 16
# stencils under the system HIP runtime and torch's.
# usage (on the box): bash probes/g_r06ar.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for P in none torch; do
  SCM_LIB=$R/probes/build/ht2/libscm.so PRE=$P ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_$P.log 2>&1
done
