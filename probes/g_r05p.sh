# Round 5 profile set of the shipped library: GPU suite, bench, kernel-trace
# stats of the bench, PMC passes of one bench step (HBM traffic, SQ counters),
# and a kernel trace of batch-1 drop-in calls (the stencil critical path).
# usage (on the box): bash probes/g_r05p.sh SET
set -e
S=${1:-r05p}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --gen-workers 1 --stencil-rows 0 --cpu-baseline-pairs 0 --extract-frames 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --stencil-rows 0 --extract-frames 0 > $O/trace_bench.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/sq1 -o run -- python3 $B > $O/sq1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o run -- python3 $B > $O/sq2.log 2>&1
ROWS=12 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/stencil_trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
