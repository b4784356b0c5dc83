set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s6
mkdir -p $O
cd $R
for v in base nosecond skeleton; do
  TAG=$v timeout -k 10 120 python -u probes/matcher_probe.py probes/build/$v/libscm.so >> $O/variants.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $R/probes/matcher_probe.py > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $R/probes/matcher_probe.py > $O/p2.log 2>&1
