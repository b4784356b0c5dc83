# Round 4: first window of a small batch (2 / 4 = default / 8 rounds, then
# 128), batch-1 latency alternating.
# usage (on the box): bash probes/g_r04x.sh SET
set -e
S=${1:-r04x}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for i in 1 2; do
  for w in 2 4 8; do
    SCM_FIRST_WINDOW=$w ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w${w}_$i.log 2>&1
  done
done
