# Round 4: watermark local estimate reading one coordinate per wave
# of the packed points: full -m gpu suite, batch-1 latency, stage
# profile, one bench.
# usage (on the box): bash probes/g_r04v.sh SET
set -e
S=${1:-r04v}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_$i.log 2>&1
done
ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile.log 2>&1
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --extract-frames 0 > $O/bench.log 2>&1
