# Round 6 (experiment): the last batch of a table run with a larger first
# window (SCM_VAR_LASTW0 rounds; fewer windows in the latency-bound tail),
# same-box bench A/B, then one run with the parity check of the last batch's
# pairs.  usage (on the box): bash probes/g_r06h.sh SET
set -e
S=${1:-r06h}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
A="--steps 5 --warmup 2 --no-cpu-baseline --cpu-baseline-pairs 0 --stencil-rows 0 --extract-frames 0 --no-isolated"
for i in 1 2; do
  for w in 0 4 8 16; do
    SCM_VAR_LASTW0=$w timeout -k 10 300 python -u bench.py $A > $O/ab_w${w}_$i.log 2>&1
  done
done
SCM_VAR_LASTW0=8 timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  --stencil-rows 0 --extract-frames 0 --no-isolated > $O/parity_w8.log 2>&1
