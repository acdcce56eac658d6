# Knob sweep of the committed kernel at the driver form (same box,
# interleaved with the default): block region, tail regions, priority mode.
# usage: bash tools/calls/gpu_r04_knobs.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
B="--steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
timeout -k 10 120 python -u bench.py $B > $O/ab_warm.json 2>/dev/null
step warm $?
for i in 1 2; do
  timeout -k 10 120 python -u bench.py $B > $O/ab_base_$i.json 2>/dev/null
  step "base $i" $?
  for k in block_region=64 block_region=128 tail=0,0.5,1 tail=0,1,0.5 tail=0,2,1 prio_mode=0 prio_mode=3; do
    n=$(echo $k | tr '=,.' '___')
    timeout -k 10 120 python -u bench.py $B --tune $k > $O/ab_${n}_$i.json 2>/dev/null
    step "$k $i" $?
  done
done
exit 0
