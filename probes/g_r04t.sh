# Round 4: point loads in flight in the replay's point loops (kLoU 4 = this
# build, 8, 16) on the table path: benches alternating (isolated verify ms).
# usage (on the box): bash probes/g_r04t.sh SET
set -e
S=${1:-r04t}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --extract-frames 0 --stencil-rows 0"
for i in 1 2; do
  timeout -k 10 300 python -u $B > $O/bench_lou4_$i.log 2>&1
  SCM_LIB=$R/probes/build/libscm_lou8.so timeout -k 10 300 python -u $B > $O/bench_lou8_$i.log 2>&1
  SCM_LIB=$R/probes/build/libscm_lou16.so timeout -k 10 300 python -u $B > $O/bench_lou16_$i.log 2>&1
done
