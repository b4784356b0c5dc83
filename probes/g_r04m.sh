# Round 4: small batches with windows of 4 rounds, then 64 (own window
# buffers): full -m gpu suite, batch-1 latency, one bench, a kernel trace of
# the stencil probe.
# usage (on the box): bash probes/g_r04m.sh SET
set -e
S=${1:-r04m}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_$i.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --extract-frames 0 > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
ROWS=12 B=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
