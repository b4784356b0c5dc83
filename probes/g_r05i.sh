# Round 5: default second F window of a small batch now 80 rounds: small-batch
# GPU tests, batch-1 latency with parallel LO in 1 / 2 windows; table path
# first windows per kind (H 4 / 8 / 16 rounds, F 2) against the default.
# usage (on the box): bash probes/g_r05i.sh SET
set -e
S=${1:-r05i}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_gpu_outcomes.py tests/test_scanner_op.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w1_$i.log 2>&1
  SCM_PARALLEL_LO_WINDOWS=2 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w2_$i.log 2>&1
done
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/ab_base_$i.log 2>&1
  SCM_TABLE_W0_H=4 timeout -k 10 300 python -u bench.py $A > $O/ab_h4_$i.log 2>&1
  SCM_TABLE_W0_H=8 timeout -k 10 300 python -u bench.py $A > $O/ab_h8_$i.log 2>&1
  SCM_TABLE_W0_H=16 timeout -k 10 300 python -u bench.py $A > $O/ab_h16_$i.log 2>&1
  SCM_TABLE_W0_F=2 timeout -k 10 300 python -u bench.py $A > $O/ab_f2_$i.log 2>&1
done
