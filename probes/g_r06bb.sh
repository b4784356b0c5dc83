# Round 6: Scanner op calls of 16 stencils under the system HIP runtime with
# AMD_DIRECT_DISPATCH=1 / =0 vs the default, three processes each.
# usage (on the box): bash probes/g_r06bb.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for i in 1 2 3; do
  ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_default_$i.log 2>&1
  AMD_DIRECT_DISPATCH=1 ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_dd1_$i.log 2>&1
  AMD_DIRECT_DISPATCH=0 ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_dd0_$i.log 2>&1
done
