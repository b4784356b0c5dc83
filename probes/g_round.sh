# GPU round check: full -m gpu suite, default bench (no CPU baseline), isolated
# matcher probe.  usage (on the box): bash probes/g_round.sh SET
set -e
S=${1:-s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
TAG=default timeout -k 10 120 python -u probes/matcher_probe.py > $O/matcher.log 2>&1
