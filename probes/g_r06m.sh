# Round 6: the matcher's small-batch column split (MatchJob tile ranges, row
# segments of 2^seg8_log2 tiles): matcher / stencil / op GPU tests, per-call
# latency at Scanner batch 1 and 2 against the previous library (HEAD build,
# probes/build/head), and a table-path bench A/B (no split there).
# usage (on the box): bash probes/g_r06m.sh SET
set -e
S=${1:-r06m}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_stencil.py \
  tests/test_scanner_op.py tests/test_gpu_golden.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  for lib in head new; do
    L=$R/probes/build/$lib/libscm.so
    [ $lib = new ] && L=$R/scanner_colmap_amd/lib/libscm.so
    for B in 1 2; do
      SCM_LIB=$L ROWS=24 B=$B timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_${lib}_b${B}_$i.log 2>&1
    done
  done
done
A="--steps 5 --warmup 2 --no-cpu-baseline --cpu-baseline-pairs 0 --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  SCM_LIB=$R/probes/build/head/libscm.so timeout -k 10 300 python -u bench.py $A > $O/ab_head_$i.log 2>&1
  timeout -k 10 300 python -u bench.py $A > $O/ab_new_$i.log 2>&1
done
