# Round 5 (diagnostics): host-side timeline of the batch-1 drop-in call --
# HIP API + kernel + copy trace of the stencil probe.
# usage (on the box): bash probes/g_r05q.sh SET
set -e
S=${1:-r05q}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ROWS=12 B=1 timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
