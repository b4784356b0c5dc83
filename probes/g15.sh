set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline > $O/trace_bench.log 2>&1
cd $R && timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1
