# Round 4: small batches start with 4-round windows and then jump to the
# largest: full -m gpu suite, batch-1 latency of this build and of a
# kMaxWindow = 64 variant (alternating), a kernel trace of the stencil probe.
# usage (on the box): bash probes/g_r04k.sh SET
set -e
S=${1:-r04k}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_new_$i.log 2>&1
  SCM_LIB=$R/probes/build/libscm_win64.so ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_win64_$i.log 2>&1
done
ROWS=24 B=1 SCM_PROFILE=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_profile.log 2>&1
cd /tmp && export TMPDIR=/tmp
ROWS=12 B=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
