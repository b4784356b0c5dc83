# N > 1 rehearsal on the 1-GPU box: GPU world-2 test, and bench.py under
# torch.distributed.run with 2 ranks sharing the GPU (gloo gather).
# usage (on the box): bash probes/g_dist.sh SET
set -e
S=${1:-s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > $O/dist_tests.log 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --images 200 --steps 2 --warmup 1 --no-cpu-baseline --extract-frames 0 --stencil-rows 0 > $O/bench_w2.log 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --dist-backend gloo --scaling strong --workload south-building-synth --steps 1 --warmup 1 --no-cpu-baseline --extract-frames 0 --stencil-rows 0 > $O/bench_w2_strong.log 2>&1
