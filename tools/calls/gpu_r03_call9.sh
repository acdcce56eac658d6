# round-3 GPU call 9: PMC A/B (one 20-frame launch per pass) of the
# perm-encoded queue build against the previous commit's build.
set -o pipefail
mkdir -p gpurun_out
FPL=20 LIBS="default tools/librt_prev.so" PASSES="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE;SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_SCA,SQ_INSTS_BRANCH,SQ_INSTS_VALU_INT32,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE" bash tools/pmc_ab.sh > gpurun_out/pmc_ab.log 2>&1 || exit 91
python tools/pmc_table.py gpurun_out > gpurun_out/pmc_table.txt 2>&1
