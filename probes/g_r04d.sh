# Round 4: drop-in batch-1 host/GPU split per call, first-window sizes.
# usage (on the box): bash probes/g_r04d.sh SET
set -e
S=${1:-r04d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for w in 0 16 8 0; do
  echo "== SCM_FIRST_WINDOW=$w" >> $O/stencil_w0.log
  ROWS=40 B=1 SCM_FIRST_WINDOW=$w timeout -k 10 200 python -u probes/stencil_probe.py >> $O/stencil_w0.log 2>&1
done
