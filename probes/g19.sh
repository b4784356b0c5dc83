set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s23
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export IMAGES=60
echo start > $O/progress.log
timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex match_tiles_i8 --output-format csv -d $O/p1 -o run -- python3 $R/probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/p1.log 2>&1
echo p1 >> $O/progress.log
timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-include-regex match_tiles_i8 --output-format csv -d $O/p2 -o run -- python3 $R/probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/p2.log 2>&1
echo p2 >> $O/progress.log
timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex match_tiles_i8 --output-format csv -d $O/p3 -o run -- python3 $R/probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/p3.log 2>&1
echo p3 >> $O/progress.log
