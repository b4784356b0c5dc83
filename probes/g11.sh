set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s14
mkdir -p $O
cd $R && timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 > $O/trace_bench.log 2>&1
