# Round 6: large batches back on one colmerge / gather workgroup per pair
# (the wide grids only for <= 256 pairs): GPU tests of the matcher, gather
# and drop-in path, batch-1 latency HEAD vs product, and the table-path A/B
# (g_r06t.sh).
# usage (on the box): bash probes/g_r06u.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_stencil.py tests/test_gpu_verify.py \
  tests/test_gpu_pipeline.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
bash probes/g_r06p.sh $S head
bash probes/g_r06t.sh $S
