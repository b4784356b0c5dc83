# GPU round profile set: GPU tests, plain bench, kernel-trace stats of the bench,
# PMC passes of one bench step (HBM traffic, SQ instruction / busy counters).
# usage (on the box): [SKIP_TESTS=1] bash probes/g_profile.sh SET
set -e
S=${1:-s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --gen-workers 1 --stencil-rows 0 --cpu-baseline-pairs 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --stencil-rows 0 > $O/trace_bench.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/sq1 -o run -- python3 $B > $O/sq1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o run -- python3 $B > $O/sq2.log 2>&1
