# Round 6: one descriptor upload per stage, the 2-D gather grid and the begin
# kernel's batched loads (probes/build/cp: the current sources), their GPU
# tests; per-call latency at batch 1 of the product build, cp and the
# second-window variants (g_r06p.sh); host-side step times of the
# SCM_DIAG_HOST_TIMES build (probes/build/ht).
# usage (on the box): bash probes/g_r06q.sh SET VARIANT...
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
SCM_LIB=$R/probes/build/cp/libscm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py \
  tests/test_gpu_stencil.py tests/test_gpu_verify.py tests/test_gpu_outcomes.py tests/test_gpu_pipeline.py \
  tests/test_scanner_op.py tests/test_gpu_golden.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > $O/tests_cp.log 2>&1
SCM_LIB=$R/probes/build/ht/libscm.so ROWS=24 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_ht.log 2>&1
bash probes/g_r06p.sh "$@"
