set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s15
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for e in 1024 2048 512; do SCM_EDGE_PAIRS=$e timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_e$e.log 2>&1; done
SCM_EDGE_PAIRS=1024 SCM_BATCH_PAIRS=6144 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_e1024_b6144.log 2>&1
