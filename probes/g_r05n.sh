# Round 5: H's solves and scores on a second scoring stream beside F's: full
# GPU suite, batch-1 latency against SCM_H_SIDE=0, a stencil kernel trace.
# usage (on the box): bash probes/g_r05n.sh SET
set -e
S=${1:-r05n}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_def_$i.log 2>&1
  SCM_H_SIDE=0 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_hmain_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
ROWS=12 B=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/stencil_probe.py > $O/stencil_trace.log 2>&1
