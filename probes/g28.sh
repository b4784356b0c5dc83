set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
B=probes/build
IMAGES=200 timeout -k 10 600 python3 probes/match_variants.py $B/libscm_bar1.so $B/libscm_bar2.so $B/libscm_bar4.so $B/libscm_bar1.so $B/libscm_bar2.so $B/libscm_bar4.so > $O/mv.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_bar2.log 2>&1
cp $B/libscm_bar4.so scanner_colmap_amd/lib/libscm.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_bar4.log 2>&1
