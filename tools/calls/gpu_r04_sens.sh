# Sensitivity A/B (timing only, no test suite): the driver-form bench of the
# in-tree build interleaved with each given variant build, 3 rounds.
# usage: bash tools/calls/gpu_r04_sens.sh <out dir> <lib> [<lib> ...]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
shift
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
B="--steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
timeout -k 10 120 python -u bench.py $B > $O/ab_warm.json 2>/dev/null
step warm $?
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py $B > $O/ab_base_$i.json 2>/dev/null
  step "base $i" $?
  for L in "$@"; do
    n=$(basename $L .so)
    timeout -k 10 120 python -u bench.py $B --lib $L > $O/ab_${n}_$i.json 2>/dev/null
    step "$n $i" $?
  done
done
exit 0
