# Round 6: kernel + HIP runtime trace of the table-path bench (when does the
# host enqueue each batch's matcher relative to the GPU timeline).
# usage (on the box): bash probes/g_r06ah.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --stencil-rows 0 --no-isolated --extract-frames 0 > $O/bench.log 2>&1
