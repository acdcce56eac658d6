# round-4 GPU call 2: the SIMD issue price of every VALU form the render
# kernel executes (tools/ubench/valu_forms, in-kernel s_memtime, at 1, 2, 4
# and 6 waves per SIMD) and which PMC class each form increments, incl.
# SQ_ACTIVE_INST_VALU2 (dual issue); then the driver-form bench with the
# run's own clock, its rocprofv3 kernel trace, and the PMC passes of one
# 20-frame launch (tools/pmc_round.sh, two new passes).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04/c2
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for w in 4 1 2 6; do
  timeout -k 10 120 tools/ubench/valu_forms $w > $O/valu_forms_w$w.txt 2>&1
  step "valu_forms w$w" $?
done
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_CVT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$R/$O/ub_pmc_$i" -o run \
      --output-format csv -- "$R/tools/ubench/valu_forms" 4 > "$R/$O/ub_pmc_$i.log" 2>&1
  step "ubench pmc $i" $?
done
cd "$R"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > $O/bench.json 2> $O/bench.err
step bench $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 \
    > "$R/$O/prof.json" 2> "$R/$O/prof.err"
step rocprof $?
cd "$R"
FPL=20 bash tools/pmc_round.sh > $O/pmc_round.log 2>&1
step pmc $?
mv gpurun_out/pmc_* $O/ 2>/dev/null
exit 0
