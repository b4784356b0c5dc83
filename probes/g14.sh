set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s17
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
IMAGES=200 timeout -k 10 300 python3 probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/mv_i8.log 2>&1
SCM_MATCH_BF16=1 IMAGES=200 timeout -k 10 300 python3 probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/mv_bf16.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
timeout -k 10 120 probes/build/score_bench > $O/score_bench.log 2>&1
SCM_PROFILE=1 SCM_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/prof.log 2>&1
