set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_q3
mkdir -p $O
cd $R
SCM_LIB=probes/build/libscm_q3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
bash probes/g_vbench.sh r03_q3 base q3 base q3
