set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_bal8192.log 2>&1
SCM_BALANCED=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_unbal.log 2>&1
SCM_BATCH_PAIRS=6144 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_bal6144.log 2>&1
SCM_BATCH_PAIRS=4096 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_bal4096.log 2>&1
SCM_BATCH_PAIRS=10000 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_bal10000.log 2>&1
