# Round 4: batch-1 drop-in after the decoupled draws -- stage cycles
# (SCM_PROFILE=1) and a rocprofv3 kernel trace of the stencil probe.
# usage (on the box): bash probes/g_r04i.sh SET
set -e
S=${1:-r04i}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile.log 2>&1
cd /tmp && export TMPDIR=/tmp
ROWS=12 B=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
