# Round 5: a small batch's second F window around 64 rounds (48 / 64 / 80 /
# 96), parallel LO of the first window on, and 64 with it off.
# usage (on the box): bash probes/g_r05h.sh SET
set -e
S=${1:-r05h}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
sha256sum scanner_colmap_amd/lib/libscm.so | cut -c1-16 > $O/lib_sha16
for i in 1 2; do
  for w in 48 64 80 96; do
    SCM_SMALL_F_W1=$w ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_fw${w}_$i.log 2>&1
  done
  SCM_SMALL_F_W1=64 SCM_PARALLEL_LO=0 ROWS=40 timeout -k 10 200 python -u probes/stencil_probe.py > $O/stencil_fw64_plo0_$i.log 2>&1
done
