set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_w16.log 2>&1
cp probes/build/libscm_win32.so scanner_colmap_amd/lib/libscm.so
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_w32.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_w32.log 2>&1
cp probes/build/libscm_win64.so scanner_colmap_amd/lib/libscm.so
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_w64.log 2>&1
SCM_BALANCED=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_w64_unbal.log 2>&1
