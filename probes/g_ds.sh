# Round 4: decoupled draws (window r's draws on their own stream beside window
# r - 1's scoring) -- full -m gpu suite on the build, then batch-1 drop-in
# latency with the draw stream on and off (SCM_DRAW_STREAM=0), alternating.
# usage (on the box): bash probes/g_ds.sh SET
set -e
S=${1:-ds}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  SCM_DRAW_STREAM=0 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_off_$i.log 2>&1
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_on_$i.log 2>&1
done
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --extract-frames 0"
SCM_LIB=$R/probes/build/libscm_base.so timeout -k 10 300 python -u $B > $O/bench_base.log 2>&1
timeout -k 10 300 python -u $B > $O/bench_new.log 2>&1
