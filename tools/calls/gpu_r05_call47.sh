# round 5: the 8K frame on one GPU (one 1024-spp frame per launch) against
# the library before the lead items (rec) and before the pipelined chunk
# loop (prev): same box, 3 rounds.  usage: bash tools/calls/gpu_r05_call47.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab8k rec=bevy_raytrace_amd/librt_hip_rec.so prev=bevy_raytrace_amd/librt_hip_prev.so cur=product -- --config rtiow8k --steps 1 --warmup 0
step ab8k $?
exit 0
