#!/bin/bash
# One rocprofv3 --pmc pass (kernel trace only) over one FPL-frame headline
# launch, for quick instruction-mix comparisons of two builds.
# usage: FPL=2 bash tools/pmc_pass.sh <out dir> "<counters>" [bench args, e.g. --lib X]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
CTR=$2
shift 2
mkdir -p "$R/$O"
cd /tmp && export TMPDIR=/tmp
FPL=${FPL:-2}
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTR -d "$R/$O/pass" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps $FPL --warmup 0 --frames-per-launch $FPL --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 0 "$@" > "$R/$O/pass.log" 2>&1
rc=$?
echo "pass ($CTR) $* rc=$rc"
exit $rc
