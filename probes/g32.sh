set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
shift
cd $R
export SCM_SERIAL=1
for v in "$@"; do
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 -c "
import sys, runpy; sys.path.insert(0, '$R'); sys.argv=['$R/bench.py','--no-cpu-baseline','--steps','1','--warmup','0']
from scanner_colmap_amd import _abi; _abi.load_library('$R/probes/build/libscm_$v.so')
runpy.run_path('$R/bench.py', run_name='__main__')" > $O/$v.log 2>&1
done
