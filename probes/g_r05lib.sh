# Round 5 (diagnostics): same-box bench A/B of a library variant
# (probes/build/$VAR.so via SCM_LIB) against the shipped build, alternating.
# usage (on the box): VAR=libscm_x bash probes/g_r05lib.sh SET
set -e
S=${1:-r05lib}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so probes/build/$VAR.so | cut -c1-16 > $O/lib_sha16
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $A > $O/ab_base_$i.log 2>&1
  SCM_LIB=$R/probes/build/$VAR.so timeout -k 10 300 python -u bench.py $A > $O/ab_var_$i.log 2>&1
done
