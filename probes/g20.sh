set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s25
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export SCM_SERIAL=1
echo start > $O/progress.log
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex rs_score --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/p1.log 2>&1
echo p1 >> $O/progress.log
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex rs_score --output-format csv -d $O/p2 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/p2.log 2>&1
echo p2 >> $O/progress.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/t.log 2>&1
