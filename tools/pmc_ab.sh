#!/bin/bash
# PMC A/B of two library builds on one box: the same counter passes over one
# FPL-frame bench launch for each build (LIBS="default tools/librt_hip_r01.so"),
# one rocprofv3 run per (pass, build), each under its own time limit; outputs
# gpurun_out/pab_<build index>_<pass>/ (tools/pmc_table.py prints the table).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
FPL=${FPL:-8}
LIBS=${LIBS:-"default tools/librt_hip_r01.so"}
PASSES=${PASSES:-"SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_WAIT_INST_LDS,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE;SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_MISC,SQ_INSTS_BRANCH,GRBM_GUI_ACTIVE"}
IFS=';' read -ra PS <<< "$PASSES"
b=0
for lib in $LIBS; do
  b=$((b+1))
  extra=""
  if [ "$lib" != default ]; then extra="--lib $R/$lib"; fi
  p=0
  for grp in "${PS[@]}"; do
    p=$((p+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${grp//,/ } -d "$R/gpurun_out/pab_${b}_${p}" -o run \
        --output-format csv -- python3 "$R/bench.py" --steps $FPL --warmup 0 --frames-per-launch $FPL \
        --no-cpu-baseline --reuse-steps 0 --cull-steps 0 $extra > "$R/gpurun_out/pab_${b}_${p}.log" 2>&1
    rc=$?
    echo "build $b ($lib) pass $p rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo PMC_AB_OK
