# Round 4: draws on the matching stream (the early final pass no longer
# queues behind them) and windows capped at the last known trial bound:
# full -m gpu suite, batch-1 latency with the draw stream on and off,
# benches of this build and the previous one alternating, a kernel trace of
# the stencil probe; batch-1 latency with kLoU = 8 / 16 point loads in flight,
# and with windows jumping to the largest size after the first (first window
# 16 (default), 8, 4, 2 rounds).
# usage (on the box): bash probes/g_r04j.sh SET
set -e
S=${1:-r04j}
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
for i in 1 2; do
  SCM_LIB=$R/probes/build/libscm_prev.so timeout -k 10 300 python -u $B > $O/bench_prev_$i.log 2>&1
  timeout -k 10 300 python -u $B > $O/bench_new_$i.log 2>&1
done
for v in lou8 lou16; do
  SCM_LIB=$R/probes/build/libscm_$v.so ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_$v.log 2>&1
done
ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_on_3.log 2>&1
for w in 0 8 4 2; do
  SCM_FIRST_WINDOW=$w SCM_LIB=$R/probes/build/libscm_jump.so ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_jump_w$w.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
ROWS=12 B=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
