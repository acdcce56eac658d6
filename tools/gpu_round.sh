#!/bin/bash
# One GPU round: smoke -> bench (headline, 4K, 10k) -> rocprofv3 kernel trace
# of the bench command (warmup = one launch of the timed size, so the rocprof
# average per render launch is the timed launch's duration) -> VALU counter
# calibration (tools/ubench/valu_busy) -> PMC passes over one 24-frame launch
# (tools/pmc_round.sh). Each GPU step has its own time limit; the first
# failure ends the call.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
step smoke $?
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
step bench $?
timeout -k 10 400 python bench.py --config rtiow4k --steps 1 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 1 --frames-per-launch 1 > gpurun_out/bench_4k.json 2>> gpurun_out/bench.err
step bench_4k $?
timeout -k 10 400 python bench.py --config spheres10k1080 --steps 2 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 2 --frames-per-launch 2 > gpurun_out/bench_10k.json 2>> gpurun_out/bench.err
step bench_10k $?
timeout -k 10 400 python bench.py --config rtiow8k --steps 1 --warmup 0 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 0 --frames-per-launch 1 > gpurun_out/bench_8k_1gpu.json 2>> gpurun_out/bench.err
step bench_8k_1gpu $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --reuse-steps 0 --warmup 24 \
    > "$R/gpurun_out/prof.log" 2>&1
step rocprof $?
cd "$R"
if [ "${CALIB:-0}" = 1 ]; then  # VALU issue calibration (tools/ubench/valu_busy, built by hand)
timeout -k 10 120 tools/ubench/valu_busy > gpurun_out/valu_busy.log 2>&1
step valu_busy $?
cd /tmp
CLS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CLS -d "$R/gpurun_out/vb_pmc" -o run \
    --output-format csv -- "$R/tools/ubench/valu_busy" > "$R/gpurun_out/vb_pmc.log" 2>&1
step vb_pmc $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CLS -d "$R/gpurun_out/rk_cls" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 24 --warmup 0 --frames-per-launch 24 \
    --no-cpu-baseline --reuse-steps 0 --cull-steps 0 > "$R/gpurun_out/rk_cls.log" 2>&1
step rk_cls $?
cd "$R"
fi
timeout -k 10 900 tools/pmc_round.sh
step pmc_round $?
echo ROUND_OK
