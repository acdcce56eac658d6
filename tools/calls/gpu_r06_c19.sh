# round 6 call 19: the final measurement record (tools/calls/gpu_r06_record.sh),
# then the headline's work chunk per atomic re-measured on the final kernel
# (knob wave_chunk, 5 rounds).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r06_record.sh $O/record
step record $?
ROUNDS=5 CONFIGS="rtiow1080" bash tools/calls/gpu_r06_ab.sh $O/chunk base=product c96=product:wave_chunk=96 c128=product:wave_chunk=128
step chunk $?
exit 0
