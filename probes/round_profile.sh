set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r01f
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r01f/fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --gen-workers 1 > $R/gpurun_out/r01f/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r01f/write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --gen-workers 1 > $R/gpurun_out/r01f/write.log 2>&1
python3 $R/profiles/pmc_summary.py $R/gpurun_out/r01f/fetch/run_counter_collection.csv $R/gpurun_out/r01f/write/run_counter_collection.csv $R/profiles/r01_pmc_match.json > $R/gpurun_out/r01f/pmc_summary.log
cp $R/profiles/r01_pmc_match.json $R/gpurun_out/r01f/
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01f/trace -o run -- python3 $R/bench.py > $R/gpurun_out/r01f/trace_bench.log 2>&1
cd $R && timeout -k 10 400 python3 bench.py > gpurun_out/r01f/bench.log 2>&1
