set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for b in ${BATCHES:-8192 9216 7168}; do
SCM_BATCH_PAIRS=$b timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$b.$RANDOM.log 2>&1
done
