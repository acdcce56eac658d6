# round 6 call 36: on top of the trackers build (the product): -O2 instead of
# -O3 (o2), and -unroll-threshold=150 (ut150) -- headline (4 rounds), 4K, 10k (3).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=4 CONFIGS="rtiow1080" bash tools/calls/gpu_r06_ab.sh $O base=product o2=tools/librt_sched3_o2.so ut150=tools/librt_sched3_ut150.so
step h $?
ROUNDS=3 CONFIGS="rtiow4k" bash tools/calls/gpu_r06_ab.sh $O base=product o2=tools/librt_sched3_o2.so ut150=tools/librt_sched3_ut150.so
step 4k $?
ROUNDS=3 CONFIGS="spheres10k1080" bash tools/calls/gpu_r06_ab.sh $O base=product o2=tools/librt_sched3_o2.so ut150=tools/librt_sched3_ut150.so
step 10k $?
exit 0
