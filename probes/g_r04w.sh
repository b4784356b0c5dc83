# Round 4: LDS-only barriers for the cross-wave counts of the point passes
# (global stores stay in flight): full -m gpu suite, batch-1 latency, stage
# profile, one bench.
# usage (on the box): bash probes/g_r04w.sh SET
set -e
S=${1:-r04w}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_$i.log 2>&1
done
ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile.log 2>&1
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --extract-frames 0 > $O/bench.log 2>&1
