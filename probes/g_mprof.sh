# Diagnostics (GPU box): isolated matcher timing of library variants
# (probes/build/<v>/libscm.so, or "cur" = the in-tree build) and SQ PMC passes
# of the matcher kernel of the first variant.  usage: bash probes/g_mprof.sh SET v1 [v2 ...]
set -e
S=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
lib() { if [ "$1" = cur ]; then echo $R/scanner_colmap_amd/lib/libscm.so; else echo $R/probes/build/$1/libscm.so; fi; }
for v in "$@"; do
  IMAGES=${IMAGES:-120} TAG=$v timeout -k 10 150 python -u probes/matcher_probe.py $(lib $v) >> $O/variants.log 2>&1
done
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  L=$(lib $1)
  P="$R/probes/matcher_probe.py $L"
  export IMAGES=40 REPS=1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/sq1 -o run -- python3 $P > $O/sq1.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o run -- python3 $P > $O/sq2.log 2>&1
  python3 $R/probes/pmc_sq.py --kernel match_g8 $O/sq1 $O/sq2 > $O/pmc_summary.txt 2>&1
fi
