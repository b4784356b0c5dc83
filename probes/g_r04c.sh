# Round 4: digit-block epilogue model (probe), drop-in batch-1 latency with the
# verification phase profile (SCM_PROFILE=1) and a kernel trace of the calls.
# usage (on the box): bash probes/g_r04c.sh SET
set -e
S=${1:-r04c}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 90 ./probes/build/mfma_shape > $O/mfma_shape.log 2>&1
ROWS=24 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_probe.log 2>&1
ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile.log 2>&1
cd /tmp && export TMPDIR=/tmp
ROWS=12 B=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
