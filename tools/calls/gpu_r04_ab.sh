# round-4 GPU A/B call: the GPU suite on the working build, then the
# driver-form bench interleaved 3 + 3 against another build of the same ABI.
# usage: bash tools/calls/gpu_r04_ab.sh <base lib> <out dir> [extra bench args]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
BASE=$1
O=$2
shift 2
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 550 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
step tests $?
B="--steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 $*"
timeout -k 10 120 python -u bench.py $B --lib $BASE > $O/ab_warm.json 2>/dev/null
step warm $?
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py $B --lib $BASE > $O/ab_base_$i.json 2>/dev/null
  step "base $i" $?
  timeout -k 10 120 python -u bench.py $B > $O/ab_new_$i.json 2>/dev/null
  step "new $i" $?
done
exit 0
