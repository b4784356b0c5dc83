# Round 5: table path A/B -- the match finalize chain (finalize, rowcheck,
# recheck) at raised wave priority (default) against SCM_PRIO_MATCH=0, and
# with the verification's latency-bound kernels raised too (SCM_PRIO_TABLE=1),
# alternating on one box.
# usage (on the box): bash probes/g_r05v.sh SET
set -e
S=${1:-r05v}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/ab_pm_$i.log 2>&1
  SCM_PRIO_MATCH=0 timeout -k 10 300 python -u bench.py $A > $O/ab_base_$i.log 2>&1
  SCM_PRIO_TABLE=1 timeout -k 10 300 python -u bench.py $A > $O/ab_pmt_$i.log 2>&1
done
