# Diagnostics (GPU box): per-call latency of the Scanner drop-in path with
# Scanner batches of B stencils, and a rocprofv3 kernel trace of the same run.
# usage: bash probes/g_stencil_trace.sh SET [B]
set -e
S=$1
B=${2:-1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
ROWS=24 B=$B timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_probe.log 2>&1
cd /tmp && export TMPDIR=/tmp
ROWS=12 B=$B timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
