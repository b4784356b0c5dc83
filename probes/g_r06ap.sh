# Round 6: table-path steps and op calls of 64 stencils under the system ROCm
# HIP runtime vs torch's bundled one (probes/table_probe.py, stencil_probe.py PRE).
# usage (on the box): bash probes/g_r06ap.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for P in none torch none torch; do
  PRE=$P timeout -k 10 200 python -u probes/table_probe.py > $O/table_$P.$(date +%s).log 2>&1
done
