#!/bin/bash
# A/B of library builds on one box (bench.py --lib, interleaved twice) and the
# VALU / MFMA counter passes of the default build over one 24-frame launch.
# usage: tools/ab_pmc.sh lib1.so [lib2.so ...]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ARGS="--no-cpu-baseline --reuse-steps 0 --cull-steps 0"
for rep in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_base_$rep.json 2>> gpurun_out/ab.err
  step "base $rep" $?
  python -c "import json;d=json.load(open('gpurun_out/ab_base_$rep.json'));print('base', d['value'], d['roofline']['kernel_ms_per_launch'])"
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    timeout -k 10 300 python bench.py $ARGS --lib "$lib" > gpurun_out/ab_${n}_$rep.json 2>> gpurun_out/ab.err
    step "$n $rep" $?
    python -c "import json;d=json.load(open('gpurun_out/ab_${n}_$rep.json'));print('$n', d['value'], d['roofline']['kernel_ms_per_launch'])"
  done
done
if [ "${PMC:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  CMD="python3 $R/bench.py --steps 24 --warmup 0 --frames-per-launch 24 --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
  i=10
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F16 GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc_$i" -o run \
        --output-format csv -- $CMD > "$R/gpurun_out/pmc_$i.log" 2>&1
    step "pmc $i" $?
  done
fi
echo AB_OK
