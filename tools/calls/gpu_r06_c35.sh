# round 6 call 35: on top of the trackers build (the product): without the
# unclustered high-register-pressure reschedule stage (nohrp; every kernel),
# without the clustered low-occupancy reschedule stage (nolow; only the
# multi-chunk kernel's code changes) -- headline (4 rounds), 4K, 10k (3).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=4 CONFIGS="rtiow1080" bash tools/calls/gpu_r06_ab.sh $O base=product nohrp=tools/librt_sched2_nohrp.so
step h $?
ROUNDS=3 CONFIGS="rtiow4k" bash tools/calls/gpu_r06_ab.sh $O base=product nohrp=tools/librt_sched2_nohrp.so
step 4k $?
ROUNDS=3 CONFIGS="spheres10k1080" bash tools/calls/gpu_r06_ab.sh $O base=product nohrp=tools/librt_sched2_nohrp.so nolow=tools/librt_sched2_nolow.so
step 10k $?
exit 0
