# round-6 measurement record of the product kernel, every BASELINE workload
# (after tools/calls/gpu_r05_pmc.sh's counters are committed, so each line carries
# its workload's record): the headline's default bench (24 frames per launch,
# with the CPU baseline), driver form (--steps 20) and the same command under
# rocprofv3 --kernel-trace --stats; rtiow4k (1 frame), spheres10k1080 (2),
# rtiow8k (the 8K frame on one GPU); the reference's own frame through the
# shim's call sequence; then the multi-rank rehearsal on this GPU
# (tools/calls/gpu_r04_multi.sh: all 8 N = 8 shards, 8 ranks through the IPC image
# path, 2 through the RCCL gather).  usage: bash tools/calls/gpu_r06_record.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
step bench_default $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > $O/bench.json 2> $O/bench.err
step bench $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 \
    > "$R/$O/prof.json" 2> "$R/$O/prof.err"
step rocprof $?
cd "$R"
timeout -k 10 400 python bench.py --config rtiow4k --steps 1 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 1 --frames-per-launch 1 > $O/bench_4k.json 2> $O/bench_other.err
step bench_4k $?
timeout -k 10 400 python bench.py --config spheres10k1080 --steps 2 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 2 --frames-per-launch 2 > $O/bench_10k.json 2>> $O/bench_other.err
step bench_10k $?
timeout -k 10 400 python bench.py --config rtiow8k --steps 1 --warmup 0 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 0 --frames-per-launch 1 > $O/bench_8k_1gpu.json 2>> $O/bench_other.err
step bench_8k_1gpu $?
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 \
    > $O/bench_reference1080.json 2> $O/bench_ref.err
step ref $?
bash tools/calls/gpu_r04_multi.sh $O/multi
step multi $?
# the driver's N>1 command shape with every rank on this one GPU (gloo
# control, IPC image path): the default line with its cross-rank row check
timeout -k 10 300 python -u bench.py --gpus 8 --same-device --dist-backend gloo --steps 20 --warmup 4 \
    > $O/multi/n8_driver_form.json 2>> $O/multi/n.err
step n8_driver_form $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step smoke $?
exit 0
