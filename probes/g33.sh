set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
