set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
B=probes/build
IMAGES=200 timeout -k 10 600 python3 probes/match_variants.py $B/libscm_base.so $B/libscm_pairbar.so $B/libscm_base.so $B/libscm_pairbar.so > $O/mv.log 2>&1
cp $B/libscm_pairbar.so scanner_colmap_amd/lib/libscm.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_pairbar.log 2>&1
