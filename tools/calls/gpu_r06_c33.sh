# round 6 call 33: scheduler options, third box: product vs trackers (trk)
# vs max-ilp on the headline (5 rounds), 4K and 10k spheres (3 rounds).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=5 CONFIGS="rtiow1080" bash tools/calls/gpu_r06_ab.sh $O base=product trk=tools/librt_sched_trk.so maxilp=tools/librt_sched_maxilp.so
step h $?
ROUNDS=3 CONFIGS="rtiow4k spheres10k1080" bash tools/calls/gpu_r06_ab.sh $O base=product trk=tools/librt_sched_trk.so maxilp=tools/librt_sched_maxilp.so
step o $?
exit 0
