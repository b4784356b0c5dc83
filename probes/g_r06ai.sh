# Round 6: the offsets upload moved ahead of the verification chain -- HIP
# runtime + kernel trace of the table-path bench, then the plain bench.
# usage (on the box): bash probes/g_r06ai.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --stencil-rows 0 --no-isolated --extract-frames 0 > $O/trace_bench.log 2>&1
cd $R
timeout -k 10 400 python3 bench.py --no-cpu-baseline --extract-frames 0 > $O/bench.log 2>&1
