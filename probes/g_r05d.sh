# Round 5: GPU suite with parallel LO in the first window only; batch-1
# latency by parallel-LO windows (off / 1 / 2); bench on this box and the
# table replay at 4 / 5 waves per SIMD (forced, with spills) and the packed
# table-path Shuffle (off: SCM_SHUFFLE_PACK=0) against it.
# usage (on the box): bash probes/g_r05d.sh SET
set -e
# (the suite runs without -x: every failure is listed; the A/B runs only if it passes)
S=${1:-r05d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  SCM_PARALLEL_LO=0 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_off_$i.log 2>&1
  SCM_PARALLEL_LO_WINDOWS=1 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w1_$i.log 2>&1
  SCM_PARALLEL_LO_WINDOWS=2 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_w2_$i.log 2>&1
done
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/ab_base_$i.log 2>&1
  SCM_SHUFFLE_PACK=0 timeout -k 10 300 python -u bench.py $A > $O/ab_nopack_$i.log 2>&1
  SCM_LIB=$R/probes/build/libscm_rp128.so timeout -k 10 300 python -u bench.py $A > $O/ab_rp128_$i.log 2>&1
  SCM_LIB=$R/probes/build/libscm_rp96.so timeout -k 10 300 python -u bench.py $A > $O/ab_rp96_$i.log 2>&1
done
