#!/bin/bash
# Memory-side PMC passes over one FPL-frame headline launch: L1 (TCP)
# accesses, misses to L2 and their latency, L2 hits / misses, LDS activity and
# the waves' wait cycles -- where the render kernel's s_waitcnt time comes
# from. One counter group per rocprofv3 run (--kernel-trace only), each under
# its own time limit. usage: FPL=2 bash tools/pmc_mem.sh <out dir> [--lib X]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
shift
mkdir -p "$R/$O"
cd /tmp && export TMPDIR=/tmp
FPL=${FPL:-2}
CMD="python3 $R/bench.py --steps $FPL --warmup 0 --frames-per-launch $FPL --no-cpu-baseline --reuse-steps 0 --cull-steps 0 $*"
i=0
for grp in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_READ_sum SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d "$R/$O/mem_$i" -o run \
      --output-format csv -- $CMD > "$R/$O/mem_$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
