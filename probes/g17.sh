set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s21
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export IMAGES=100
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-include-regex match_tiles_i8 --output-format csv -d $O/p1 -o run -- python3 $R/probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --kernel-include-regex match_tiles_i8 --output-format csv -d $O/p2 -o run -- python3 $R/probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/p2.log 2>&1
