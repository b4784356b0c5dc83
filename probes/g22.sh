set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_base.log 2>&1
SCM_HEAD_PAIRS=1024 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_h1024.log 2>&1
SCM_HEAD_PAIRS=2048 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_h2048.log 2>&1
SCM_HEAD_PAIRS=1024 SCM_BATCH_PAIRS=4096 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_h1024_b4096.log 2>&1
SCM_HEAD_PAIRS=2048 SCM_BATCH_PAIRS=6144 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_h2048_b6144.log 2>&1
SCM_HEAD_PAIRS=1024 SCM_BATCH_PAIRS=12288 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_h1024_b12288.log 2>&1
