# Round 4: kMaxWindow = 64 (windows up to 4,096 trials) on the table path:
# benches of this build (32) and the win64 variant, alternating.
# usage (on the box): bash probes/g_r04l.sh SET
set -e
S=${1:-r04l}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --extract-frames 0"
for i in 1 2; do
  timeout -k 10 300 python -u $B > $O/bench_w32_$i.log 2>&1
  SCM_LIB=$R/probes/build/libscm_win64.so timeout -k 10 300 python -u $B > $O/bench_w64_$i.log 2>&1
done
