# round 5: one tail for every launch (the N = 8 shard's 1,1,0.25 rule
# dropped): the shard / image-out parity tests on both builds, all 8 shards
# against the full frame (tools/calls/gpu_r04_multi.sh: shard_all + the 8-rank IPC
# rehearsal, hashes against N = 1).  usage: bash tools/calls/gpu_r05_call53.sh <relative out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -k "shard or image_out or schedule or tail" -x -q --timeout 250 --timeout-method thread > $O/t.log 2>&1
step tests $?
timeout -k 10 400 python -u -m pytest tests -m gpu -k "shard or image_out or schedule or tail" -x -q --timeout 250 --timeout-method thread --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/tc.log 2>&1
step tests_checked $?
bash tools/calls/gpu_r04_multi.sh $O/multi
step multi $?
exit 0
