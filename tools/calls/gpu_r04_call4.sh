# round-4 GPU call 4: the committed kernel's measurement record -- the
# driver-form bench, its rocprofv3 kernel trace (the bench line inside the
# profiled run carries that run's own clock), a memory-latency PMC pass
# (Little's law per instruction class, instruction fetch); the reference's
# own frame through the shim's call sequence at both depths (1 and 2 renders
# in flight); the IPC image path's collect on one GPU (2 ranks) under the
# kernel trace, write-through + release vs the RCCL-gather collect.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04/c4
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > $O/bench.json 2> $O/bench.err
step bench $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 \
    > "$R/$O/prof.json" 2> "$R/$O/prof.err"
step rocprof $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_IFETCH SQ_IFETCH_LEVEL GRBM_GUI_ACTIVE \
    -d "$R/$O/pmc_lat" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 0 --frames-per-launch 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 \
    > "$R/$O/pmc_lat.log" 2>&1
step pmc_lat $?
cd "$R"
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > $O/bench_reference1080.json 2> $O/bench_ref.err
step bench_ref1080 $?
cd /tmp
for g in ipc rccl; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/n2_$g" -o run --output-format csv \
      -- python3 "$R/bench.py" --gpus 2 --same-device --dist-backend gloo --gather $g --steps 20 --warmup 4 \
      --no-cpu-baseline --reuse-steps 0 --cull-steps 0 > "$R/$O/n2_$g.json" 2> "$R/$O/n2_$g.err"
  step "n2 $g" $?
done
exit 0
