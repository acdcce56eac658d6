# round-3 GPU call 22: the measurement record of the final round-3 kernel --
# PMC passes over one 20-frame launch (tools/pmc_round.sh FPL=20) summarised
# into profiles/ (copied to gpurun_out/), then the driver-form bench reading
# that record, a rocprofv3 kernel trace of the same form, and the GPU suite.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
FPL=20 bash tools/pmc_round.sh > gpurun_out/pmc_round.log 2>&1
step pmc $?
python3 tools/pmc_summary.py gpurun_out r03 rtiow1080 20 > gpurun_out/pmc_summary.log 2>&1
step pmc_summary $?
cp profiles/r03_pmc_rtiow1080.json profiles/pmc_traffic.json gpurun_out/
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err
step bench $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 \
    > "$R/gpurun_out/prof.json" 2> "$R/gpurun_out/prof.err"
step rocprof $?
cd "$R"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread --durations=25 > gpurun_out/gpu_tests.log 2>&1
step tests $?
