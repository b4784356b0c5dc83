# A/B of verifier scoring variants (short benches, alternating order) + the
# verification GPU tests on the variant.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r03_vm
SCM_LIB=probes/build/libscm_smfma.so timeout -k 10 400 python -u -m pytest tests/test_gpu_outcomes.py tests/test_gpu_verify.py tests/test_gpu_stencil.py tests/test_gpu_golden.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_vm/tests.log 2>&1
bash probes/g_vbench.sh r03_vm vbase smfma vbase smfma
