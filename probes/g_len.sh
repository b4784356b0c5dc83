# Throughput against table length (the drain at the end of each table run):
# default bench workload with 1000, 2000 and 4000 images per table run.
# usage (on the box): bash probes/g_len.sh SET
set -e
S=${1:-len}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for n in 1000 2000 4000; do
  timeout -k 10 300 python -u bench.py --images $n --steps 2 --warmup 1 --no-cpu-baseline --stencil-rows 0 --extract-frames 0 --no-isolated > $O/bench_$n.log 2>&1
done
