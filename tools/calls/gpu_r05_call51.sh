# round 5, final: the GPU suite on both builds + smoke, then the record.
# usage: bash tools/calls/gpu_r05_call51.sh <relative out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_tests.sh $1/tests
step tests $?
bash tools/calls/gpu_r05_record.sh $1/record
step record $?
exit 0
