# Round 6: Scanner op calls of 16 and 64 stencils under the system HIP runtime
# with ROC_ACTIVE_WAIT_TIMEOUT raised (the runtime's active-wait window before
# it sleeps on the completion interrupt), after a first plain process.
# usage (on the box): bash probes/g_r06be.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_first.log 2>&1
for i in 1 2; do
  ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_plain_$i.log 2>&1
  ROC_ACTIVE_WAIT_TIMEOUT=100000 ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_aw_$i.log 2>&1
  ROC_ACTIVE_WAIT_TIMEOUT=100000 ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_aw_$i.log 2>&1
done
