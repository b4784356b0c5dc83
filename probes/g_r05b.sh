# Round 5: GPU suite on the merged fp32 watermark RANSAC (+ index vector in the
# H area), the fix's teeth (variant with the vector back in the F area), and
# an A/B of the table path's batch schedule / stream priority.
# usage (on the box): bash probes/g_r05b.sh SET
set -e
S=${1:-r05b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -s > $O/tests.log 2>&1
SCM_LIB=$R/probes/build/libscm_fsidx.so timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_stencil.py -k watermark_index_vector > $O/teeth.log 2>&1 || echo "teeth rc $?" >> $O/teeth.log
A="--no-cpu-baseline --stencil-rows 0 --extract-frames 0 --no-isolated --steps 5"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/ab_base_$i.log 2>&1
  SCM_BATCH_SMALL_FIRST=1 timeout -k 10 300 python -u bench.py $A > $O/ab_small_$i.log 2>&1
  SCM_MATCH_PRIO=high timeout -k 10 300 python -u bench.py $A > $O/ab_mprio_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
SCM_BATCH_SMALL_FIRST=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_small -o run -- python3 $R/bench.py $A > $O/trace_small.log 2>&1
