set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export SCM_SERIAL=1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/base.log 2>&1
cd $R
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/noslow -o run -- python3 -c "
import sys, runpy; sys.argv=['bench.py','--no-cpu-baseline','--steps','1','--warmup','0']
from scanner_colmap_amd import _abi; _abi.load_library('probes/build/libscm_noslow.so')
runpy.run_path('bench.py', run_name='__main__')" > $O/noslow.log 2>&1
