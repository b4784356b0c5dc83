# Round profile set (run on the GPU box via gpurun): GPU tests, PMC HBM traffic
# passes of the matcher (summarised here afterwards by profiles/pmc_summary.py,
# profiles/ does not travel), kernel-trace stats of the default bench, plain bench.
# usage: bash probes/round_profile.sh SET KERNEL   (e.g. r01g match_tiles_i8_kernel)
set -e
SET=${1:-r01g}
KERNEL=${2:-match_tiles_i8_kernel}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$SET
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --gen-workers 1 > $O/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --gen-workers 1 > $O/write.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline > $O/trace_bench.log 2>&1
cd $R && timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1
