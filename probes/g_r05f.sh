# Round 5: skewed wave-Shuffle lane tables + pass-level wave draws (small
# batches), packed table Shuffle removed: full GPU suite, batch-1 latency
# (parallel LO off / first window), stage profile, bench.
# usage (on the box): bash probes/g_r05f.sh SET
set -e
S=${1:-r05f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  SCM_PARALLEL_LO=0 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_off_$i.log 2>&1
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w1_$i.log 2>&1
done
SCM_PARALLEL_LO=0 ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile.log 2>&1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
