# A/B of verifier occupancy variants (short benches, alternating order).
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash probes/g_vbench.sh r03_vq vbase hm2w6 w5 hm3w5 rp3 rp4 vbase hm2w6 w5 hm3w5 rp3 rp4
