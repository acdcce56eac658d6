# round-4 measurement record of the working kernel: the default bench (24
# frames per launch, with the CPU baseline), the driver-form bench (20), its
# rocprofv3 kernel trace (the profiled run's own bench line carries its
# clock), and the PMC passes of one 20-frame launch (tools/pmc_round.sh).
# usage: bash tools/calls/gpu_r04_record.sh <out dir>
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
FPL=20 bash tools/pmc_round.sh > $O/pmc_round.log 2>&1
step pmc $?
mv gpurun_out/pmc_* $O/ 2>/dev/null
exit 0
