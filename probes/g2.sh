set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
cd $R
SCM_PROFILE=1 SCM_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/profile.log 2>&1
cd /tmp
SCM_SERIAL=1 timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --gen-workers 4 > $O/pmc1.log 2>&1
