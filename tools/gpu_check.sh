#!/bin/bash
# One GPU call: the -m gpu suite, the default bench line, and (VALU=1) the
# VALU counter calibration (tools/ubench/valu_busy under rocprofv3 PMC, plus
# the same counters over one 4-frame render launch). Every GPU step has its
# own time limit; the first failure ends the call.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
  step pytest $?
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  step bench $?
  cat gpurun_out/bench.json
fi
if [ -n "${AB:-}" ]; then  # extra bench lines: AB="--tune wg_per_cu=6;--config rtiow4k ..."
  IFS=';' read -ra ABS <<< "$AB"
  i=0
  for a in "${ABS[@]}"; do
    i=$((i+1))
    timeout -k 10 400 python bench.py --no-cpu-baseline --reuse-steps 0 --cull-steps 0 $a \
        > gpurun_out/ab_$i.json 2>> gpurun_out/ab.err
    step "ab $i ($a)" $?
    cat gpurun_out/ab_$i.json
  done
fi
if [ "${VALU:-0}" = 1 ]; then
  timeout -k 10 120 tools/ubench/valu_busy > gpurun_out/valu_busy.log 2>&1
  step valu_busy $?
  cat gpurun_out/valu_busy.log
  cd /tmp && export TMPDIR=/tmp
  CNT="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT -d "$R/gpurun_out/vb_pmc" -o run \
      --output-format csv -- "$R/tools/ubench/valu_busy" > "$R/gpurun_out/vb_pmc.log" 2>&1
  step vb_pmc $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT -d "$R/gpurun_out/rk_pmc" -o run \
      --output-format csv -- python3 "$R/bench.py" --steps 4 --warmup 0 --frames-per-launch 4 \
      --no-cpu-baseline --reuse-steps 0 --cull-steps 0 > "$R/gpurun_out/rk_pmc.log" 2>&1
  step rk_pmc $?
fi
echo ALL_OK
