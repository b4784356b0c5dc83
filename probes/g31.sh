set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
SCM_PROFILE=1 SCM_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/prof.log 2>&1
