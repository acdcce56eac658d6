#!/bin/bash
# PMC passes over the headline bench command (one counter group per rocprofv3
# run, --kernel-trace only; no sys/runtime trace with --pmc), each pass under
# its own time limit. The command renders exactly one FPL-frame launch
# (--steps FPL --warmup 0; FPL=24 = the default bench launch) of workload CFG
# (default rtiow1080). Output under $OUT/pmc_* (default gpurun_out);
# tools/pmc_summary.py <OUT> <tag> <CFG> <FPL> turns it into profiles/.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$(realpath -m "${OUT:-$R/gpurun_out}")  # absolute: the passes run from /tmp
cd /tmp && export TMPDIR=/tmp
FPL=${FPL:-24}
CFG=${CFG:-rtiow1080}
mkdir -p "$OUT"
CMD="python3 $R/bench.py --config $CFG --steps $FPL --warmup 0 --frames-per-launch $FPL --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F16 GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_CVT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/pmc_$i" -o run \
      --output-format csv -- $CMD > "$OUT/pmc_$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
