set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s16
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
IMAGES=200 timeout -k 10 300 python3 probes/match_variants.py probes/build/libscm_cur.so probes/build/libscm_skel.so > $O/mv.log 2>&1
cd /tmp && export TMPDIR=/tmp
IMAGES=460 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o run -- python3 $R/probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/new.log 2>&1
