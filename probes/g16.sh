set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s27
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
IMAGES=200 timeout -k 10 300 python3 probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/mv_i8.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
