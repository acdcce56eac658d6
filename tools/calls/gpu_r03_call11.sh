# round-3 GPU call 11: the pixel-major kernel's measurement record -- the
# driver-form bench (--steps 20), a rocprofv3 kernel trace of the same form
# (warmup = one launch of the timed size), and the PMC passes over one
# 20-frame launch (tools/pmc_round.sh FPL=20).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err
step bench $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 \
    > "$R/gpurun_out/prof.json" 2> "$R/gpurun_out/prof.err"
step rocprof $?
cd "$R"
FPL=20 bash tools/pmc_round.sh > gpurun_out/pmc_round.log 2>&1
step pmc $?
