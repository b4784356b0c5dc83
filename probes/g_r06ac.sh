# Round 6: the Scanner drop-in path over op batch sizes 1-32 (bench drop-in
# legs only: the table step kept short) on the shipped library, and the head
# of round 6 (probes/build/head) for batch 1-8.
# usage (on the box): bash probes/g_r06ac.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
A="--steps 1 --warmup 1 --no-cpu-baseline --cpu-baseline-pairs 0 --extract-frames 0 --no-isolated"
timeout -k 10 400 python -u bench.py $A --stencil-batches 1:128,2:128,4:128,8:128,16:256,32:256 > $O/legs_new.log 2>&1
SCM_LIB=$R/probes/build/head/libscm.so timeout -k 10 400 python -u bench.py $A --stencil-batches 1:128,2:128,4:128,8:128 > $O/legs_head.log 2>&1
