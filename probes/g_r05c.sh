# Round 5: GPU suite with the parallel-LO replay of small batches and the
# chunked table runs; batch-1 latency A/B (parallel LO on / off); bench; the
# 2-rank gloo rehearsal with the gather inside the step vs across steps.
# usage (on the box): bash probes/g_r05c.sh SET
set -e
S=${1:-r05c}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  for p in 1 0; do
    SCM_PARALLEL_LO=$p ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_plo${p}_$i.log 2>&1
  done
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
for g in chunked step; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --gather $g --images 300 --steps 3 --warmup 1 --no-cpu-baseline --extract-frames 0 --stencil-rows 0 --no-isolated > $O/dist_w2_$g.log 2>&1
done
