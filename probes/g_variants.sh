# Diagnostics (GPU box): isolated matcher timing of the libscm.so variants
# built by probes/build_match_variants.sh.  usage: bash probes/g_variants.sh SET v1 v2 ...
set -e
S=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
for v in "$@"; do
  IMAGES=${IMAGES:-120} TAG=$v timeout -k 10 150 python -u probes/matcher_probe.py probes/build/$v/libscm.so >> $O/variants.log 2>&1
done
