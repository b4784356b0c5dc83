# Per-kernel time of the default bench, serial (SCM_SERIAL=1) and overlapped.
# usage (on the box): bash probes/g_serial.sh SET
set -e
S=${1:-s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export SCM_SERIAL=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- python3 $R/bench.py --no-cpu-baseline --stencil-rows 0 --cpu-baseline-pairs 0 > $O/serial.log 2>&1
unset SCM_SERIAL
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --stencil-rows 0 --cpu-baseline-pairs 0 > $O/trace.log 2>&1
