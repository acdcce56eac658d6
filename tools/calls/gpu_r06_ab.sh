# round 6 A/B call: optionally the GPU suite (--tests), then for each workload
# in CONFIGS (default rtiow1080) the driver-form bench (--steps 20 for the
# headline; the workload's own default otherwise) interleaved over the arms,
# ROUNDS rounds (default 3).  usage:
#   CONFIGS="rtiow1080 spheres10k1080" bash tools/calls/gpu_r06_ab.sh <out dir> [--tests] <arm>=<lib|product>[:knob=v,...] ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
shift
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
TESTS=0
ARMS=()
for a in "$@"; do
  if [ "$a" = --tests ]; then TESTS=1; else ARMS+=("$a"); fi
done
if [ $TESTS -eq 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
  step tests $?
  tail -2 $O/gpu_tests.log
fi
armargs() {
  local spec=${1#*=} lib tunes out=""
  lib=${spec%%:*}
  if [ "$lib" != product ]; then out="--lib $lib"; fi
  if [ "$spec" != "$lib" ]; then
    tunes=${spec#*:}
    for kv in ${tunes//,/ }; do out="$out --tune ${kv//\//,}"; done
  fi
  echo "$out"
}
for cfg in ${CONFIGS:-rtiow1080}; do
  case $cfg in
    rtiow1080) B="--steps 20 --warmup 4" ;;
    spheres10k1080) B="--steps 2 --warmup 2 --frames-per-launch 2" ;;
    *) B="--steps 1 --warmup 1 --frames-per-launch 1" ;;
  esac
  B="$B --config $cfg --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
  mkdir -p $O/$cfg
  timeout -k 10 200 python -u bench.py $B $(armargs ${ARMS[0]}) > $O/$cfg/ab_warm.json 2>/dev/null
  step "warm $cfg" $?
  for i in $(seq 1 ${ROUNDS:-3}); do
    for a in "${ARMS[@]}"; do
      timeout -k 10 200 python -u bench.py $B $(armargs $a) > $O/$cfg/ab_${a%%=*}_$i.json 2>$O/$cfg/ab_${a%%=*}_$i.err
      step "$cfg ${a%%=*} $i" $?
    done
  done
  python tools/ab_table.py $O/$cfg | tail -3
done
exit 0
