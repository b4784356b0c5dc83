set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s12
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ldsm noldsm; do
  IMAGES=460 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/probes/match_variants.py --one=$R/probes/build/libscm_$v.so > $O/$v.log 2>&1
done
cd $R && SCM_PROFILE=1 IMAGES=460 timeout -k 10 300 python3 probes/match_variants.py --one=$R/probes/build/libscm_noldsm.so > $O/prof.log 2>&1
