# Round 6: HIP runtime + kernel + copy trace of Scanner op calls of 64
# stencils (where the host waits inside a call).
# usage (on the box): bash probes/g_r06al.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ROWS=320 B=64 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
