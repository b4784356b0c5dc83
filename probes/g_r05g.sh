# Round 5: per-kind window sizes -- a small batch's second F window of 128
# (default) / 64 / 32 rounds, parallel LO of the first window on and off;
# full GPU suite on the library.
# usage (on the box): bash probes/g_r05g.sh SET
set -e
S=${1:-r05g}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  for w in 0 64 32; do
    SCM_SMALL_F_W1=$w ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_fw${w}_$i.log 2>&1
  done
  SCM_SMALL_F_W1=32 SCM_PARALLEL_LO=0 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_fw32_plo0_$i.log 2>&1
done
SCM_SMALL_F_W1=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_stencil.py tests/test_scanner_op.py -x -v --timeout 200 --timeout-method thread > $O/tests_fw32.log 2>&1
