# GPU SIFT extraction tests (and optionally the bench's extraction leg).
# usage (on the box): bash probes/g_sift.sh SET
set -e
S=${1:-s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_sift.py -x -v --timeout 200 --timeout-method thread > $O/sift_tests.log 2>&1
