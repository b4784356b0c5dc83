set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
export SCM_BALANCED=0
for rep in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_w16_$rep.log 2>&1
LD=probes/build/libscm_win32.so timeout -k 10 300 python -c "
import sys, runpy; sys.argv=['bench.py','--no-cpu-baseline']
from scanner_colmap_amd import _abi; _abi.load_library('probes/build/libscm_win32.so')
runpy.run_path('bench.py', run_name='__main__')" > $O/b_w32_$rep.log 2>&1
timeout -k 10 300 python -c "
import sys, runpy; sys.argv=['bench.py','--no-cpu-baseline']
from scanner_colmap_amd import _abi; _abi.load_library('probes/build/libscm_win64.so')
runpy.run_path('bench.py', run_name='__main__')" > $O/b_w64_$rep.log 2>&1
done
