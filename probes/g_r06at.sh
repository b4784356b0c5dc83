# Round 6: host waits by polling (host_wait_event) -- Scanner op calls of 1,
# 16 and 64 stencils under the system HIP runtime (three processes each) and
# torch's.
# usage (on the box): bash probes/g_r06at.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for i in 1 2 3; do
  ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_none_$i.log 2>&1
  ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_none_$i.log 2>&1
  ROWS=64 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b1_none_$i.log 2>&1
done
PRE=torch ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_torch.log 2>&1
PRE=torch ROWS=320 B=64 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b64_torch.log 2>&1
PRE=torch ROWS=64 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b1_torch.log 2>&1
