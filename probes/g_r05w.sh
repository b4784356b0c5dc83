# Round 5: table path A/B -- matcher wave priority (SCM_PRIO_MATCHER: 1 every
# launch, 2 the run's last batch only) against the default (none),
# alternating on one box.
# usage (on the box): bash probes/g_r05w.sh SET
set -e
S=${1:-r05w}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/ab_base_$i.log 2>&1
  SCM_PRIO_MATCHER=1 timeout -k 10 300 python -u bench.py $A > $O/ab_all_$i.log 2>&1
  SCM_PRIO_MATCHER=2 timeout -k 10 300 python -u bench.py $A > $O/ab_last_$i.log 2>&1
done
