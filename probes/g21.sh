set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
SCM_PROFILE=1 SCM_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/prof.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && SCM_SERIAL=1 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/t.log 2>&1
