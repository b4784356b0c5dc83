set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s2/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2/b8192.log 2>&1
SCM_BATCH_PAIRS=4096 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2/b4096.log 2>&1
SCM_BATCH_PAIRS=2048 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2/b2048.log 2>&1
