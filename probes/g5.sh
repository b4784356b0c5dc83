set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export IMAGES=100
timeout -s KILL 120 rocprofv3 --kernel-include-regex "rs_score|rs_replay|match_tiles" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --output-format csv -d $O/p1 -o run -- python3 $R/probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-include-regex "rs_score|rs_replay|match_tiles" --pmc SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/p2 -o run -- python3 $R/probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-include-regex "rs_score|rs_replay|match_tiles" --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU --output-format csv -d $O/p3 -o run -- python3 $R/probes/match_variants.py --one=$R/scanner_colmap_amd/lib/libscm.so > $O/p3.log 2>&1
