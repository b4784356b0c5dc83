# Round 6: Scanner op calls of 64 and 256 stencils with the call's pairs cut
# into 1, 2 or 3 pipelined batches (SCM_BATCH_PAIRS).
# usage (on the box): bash probes/g_r06ak.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for BP in 8192 608 406; do
  SCM_BATCH_PAIRS=$BP ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_bp$BP.log 2>&1
done
for BP in 8192 2432 1622; do
  SCM_BATCH_PAIRS=$BP ROWS=1024 B=256 timeout -k 10 300 python -u probes/stencil_probe.py > $O/b256_bp$BP.log 2>&1
done
