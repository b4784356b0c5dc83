# Round-4 first check: micro-probes (i8 MFMA shapes, H split pass forms),
# the full -m gpu suite, smoke, default bench, the N > 1 rehearsal.
# usage (on the box): bash probes/g_r04a.sh SET
set -e
S=${1:-r04a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 60 ./probes/build/mfma_shape > $O/mfma_shape.log 2>&1
timeout -k 10 120 ./probes/build/hsplit_bench > $O/hsplit.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline --stencil-rows 0 --extract-frames 0 > $O/dist_bench.log 2>&1
