# Round 6: Scanner op calls of 64 stencils unprofiled, with the copy engines
# (default) and with blit-kernel copies only (HSA_ENABLE_SDMA=0), twice each.
# usage (on the box): bash probes/g_r06am.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for i in 1 2; do
  ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_sdma_$i.log 2>&1
  HSA_ENABLE_SDMA=0 ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_nosdma_$i.log 2>&1
done
