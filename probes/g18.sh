set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s38
mkdir -p $O
cd $R
B=probes/build
IMAGES=200 timeout -k 10 600 python3 probes/match_variants.py $B/libscm_base.so $B/libscm_dmerge.so $B/libscm_dmergenobar.so > $O/mv.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
