# Round 6: HIP runtime log (AMD_LOG_LEVEL=4, AMD_LOG_MASK all) of Scanner op
# calls of 16 stencils under the system runtime, after a first plain process.
# usage (on the box): bash probes/g_r06bc.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_first.log 2>&1
ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_second.log 2>&1
AMD_LOG_LEVEL=4 ROWS=64 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_log.txt 2>&1
gzip -f $O/b16_log.txt
