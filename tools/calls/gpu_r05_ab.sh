# round-5 A/B call: optionally the GPU suite on the product build, then the
# driver-form bench (--steps 20) interleaved over several builds of the same
# ABI, ROUNDS rounds (default 3).  usage:
#   bash tools/calls/gpu_r05_ab.sh <out dir> [--tests] <arm>=<lib|product>[:knob=v,knob=v] ... [-- extra bench args]
# (a value holding commas is written with '/': tail=0/0.5/1)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
shift
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
TESTS=0
ARMS=()
while [ $# -gt 0 ]; do
  case "$1" in
    --tests) TESTS=1 ;;
    --) shift; break ;;
    *) ARMS+=("$1") ;;
  esac
  shift
done
if [ $TESTS -eq 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
  step tests $?
fi
B="--steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 $*"
# arm spec name=lib[:k=v,k=v] -> bench.py arguments (--lib, --tune)
armargs() {
  local spec=${1#*=} lib tunes out=""
  lib=${spec%%:*}
  if [ "$lib" != product ]; then out="--lib $lib"; fi
  if [ "$spec" != "$lib" ]; then
    tunes=${spec#*:}
    for kv in ${tunes//,/ }; do out="$out --tune ${kv//\//,}"; done  # '/' in a value: ','  (tail=0/1/1)
  fi
  echo "$out"
}
first=${ARMS[0]}
timeout -k 10 200 python -u bench.py $B $(armargs $first) > $O/ab_warm.json 2>/dev/null
step warm $?
for i in $(seq 1 ${ROUNDS:-3}); do
  for a in "${ARMS[@]}"; do
    timeout -k 10 200 python -u bench.py $B $(armargs $a) > $O/ab_${a%%=*}_$i.json 2>$O/ab_${a%%=*}_$i.err
    step "${a%%=*} $i" $?
  done
done
exit 0
