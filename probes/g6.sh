set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s7
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
for v in v1 v2; do
  IMAGES=460 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/probes/match_variants.py --one=$R/probes/build/libscm_$v.so > $O/$v.log 2>&1
done
