# Round 6: Scanner op calls of 1 / 16 / 64 / 256 stencils under the system ROCm
# HIP runtime (PRE=none) vs torch's bundled one (PRE=torch).
# usage (on the box): bash probes/g_r06aq.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for P in none torch; do
  PRE=$P ROWS=64 B=1 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b1_$P.log 2>&1
  PRE=$P ROWS=96 B=16 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b16_$P.log 2>&1
  PRE=$P ROWS=768 B=256 timeout -k 10 200 python -u probes/stencil_probe.py > $O/b256_$P.log 2>&1
done
