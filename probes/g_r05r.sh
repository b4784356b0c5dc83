# Round 5: table path A/B -- the latency-bound kernels (replay, draws,
# shuffles, final) at raised wave priority
# (SCM_PRIO_TABLE=1) against the default, alternating on one box.
# usage (on the box): bash probes/g_r05r.sh SET
set -e
S=${1:-r05r}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/ab_base_$i.log 2>&1
  SCM_PRIO_TABLE=1 timeout -k 10 300 python -u bench.py $A > $O/ab_prio_$i.log 2>&1
done
