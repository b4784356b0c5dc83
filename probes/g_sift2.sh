# SIFT extraction: GPU tests, timing with the context's streams and with
# streams of its own (SCM_SIFT_OWN_STREAMS=1), kernel trace.
# usage (on the box): bash probes/g_sift2.sh SET [notest]
set -e
S=${1:-s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
if [ "${2:-}" != "notest" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_sift.py -x -v --timeout 200 --timeout-method thread > $O/sift_tests.log 2>&1
fi
timeout -k 10 300 python -u probes/sift_probe.py 1080 1920 16 > $O/probe_1080p.log 2>&1
SCM_SIFT_OWN_STREAMS=1 timeout -k 10 300 python -u probes/sift_probe.py 1080 1920 16 > $O/probe_1080p_own.log 2>&1
timeout -k 10 300 python -u probes/sift_probe.py 2304 3072 8 > $O/probe_3072.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/sift_probe.py 1080 1920 16 > $O/trace.log 2>&1
