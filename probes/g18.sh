set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s48
mkdir -p $O
cd $R
B=probes/build
IMAGES=200 timeout -k 10 600 python3 probes/match_variants.py $B/libscm_base.so $B/libscm_prio.so $B/libscm_base.so $B/libscm_prio.so > $O/mv.log 2>&1
