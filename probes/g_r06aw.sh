# Round 6: the box's CPU share (cgroup cpu.max, affinity) and Scanner op calls
# of 16 stencils under the system HIP runtime, plain and pinned to 8 CPUs.
# usage (on the box): bash probes/g_r06aw.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
{ cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max"; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null || true; } > $O/cpu.txt 2>&1
for i in 1 2 3; do
  ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_plain_$i.log 2>&1
  ROWS=96 B=16 timeout -k 10 200 taskset -c 0-7 python -u probes/stencil_probe.py > $O/b16_cpu8_$i.log 2>&1
done
cat /sys/fs/cgroup/cpu.stat >> $O/cpu.txt 2>/dev/null || true
