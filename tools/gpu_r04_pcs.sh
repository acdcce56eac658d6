# Stall attribution of the render kernel by PC sampling (rocprofv3 beta):
# the available sampling configurations, then stochastic cycle sampling of one
# 2-frame headline launch (each sample: the wave's PC, whether it issued, and
# why not). Summarised by tools/pcs_summary.py.
# usage: bash tools/gpu_r04_pcs.sh <out dir> [interval]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
IV=${2:-65536}
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/$O/list.txt" 2>&1
step list $?
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
    --pc-sampling-unit cycles --pc-sampling-interval $IV --kernel-trace \
    -d "$R/$O/pcs" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --frames-per-launch 2 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 0 --shim-frames 0 > "$R/$O/pcs.json" 2> "$R/$O/pcs.err"
step pcs $?
exit 0
