# round 6 call 22: work chunk sweep on the final kernel -- headline 128 (the
# rule) / 192 / 256; rtiow4k, spheres10k1080 and the 8K frame 64 (the rule)
# against 128 (round 5 measured 128 slower there, before the 4K launch had
# the s_setprio rotation).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=4 CONFIGS="rtiow1080" bash tools/calls/gpu_r06_ab.sh $O base=product c192=product:wave_chunk=192 c256=product:wave_chunk=256
step h $?
ROUNDS=4 CONFIGS="rtiow4k spheres10k1080" bash tools/calls/gpu_r06_ab.sh $O base=product c128=product:wave_chunk=128
step o $?
ROUNDS=2 CONFIGS="rtiow8k" bash tools/calls/gpu_r06_ab.sh $O base=product c128=product:wave_chunk=128
step 8k $?
exit 0
