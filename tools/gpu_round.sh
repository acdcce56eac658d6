#!/bin/bash
# One GPU round: smoke -> bench -> rocprofv3 kernel trace of the bench command
# (warmup = one launch of the timed size, so the rocprof average per render
# launch is the timed launch's duration).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 400 python bench.py --config rtiow4k --steps 1 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 1 --frames-per-launch 1 > gpurun_out/bench_4k.json 2>> gpurun_out/bench.err
timeout -k 10 400 python bench.py --config spheres10k1080 --steps 2 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 2 --frames-per-launch 2 > gpurun_out/bench_10k.json 2>> gpurun_out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --reuse-steps 0 --warmup 24 \
    > "$R/gpurun_out/prof.log" 2>&1
echo done
