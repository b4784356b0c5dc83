# SIFT extraction timing + kernel trace.  usage (on the box): bash probes/g_sift_prof.sh SET
set -e
S=${1:-s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 300 python -u probes/sift_probe.py 1080 1920 16 > $O/probe_1080p.log 2>&1
timeout -k 10 300 python -u probes/sift_probe.py 2304 3072 8 > $O/probe_3072.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/probes/sift_probe.py 1080 1920 16 > $O/trace.log 2>&1
