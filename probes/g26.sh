set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
shift
for v in "$@"; do
  if [ "$v" = base ]; then
    timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$v.log 2>&1
  else
    timeout -k 10 300 python -c "
import sys, runpy; sys.argv=['bench.py','--no-cpu-baseline']
from scanner_colmap_amd import _abi; _abi.load_library('probes/build/libscm_$v.so')
runpy.run_path('bench.py', run_name='__main__')" > $O/b_$v.log 2>&1
  fi
done
