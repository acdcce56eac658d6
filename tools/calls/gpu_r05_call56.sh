# round 5: the work chunk by the call (128 items at >= 4 pixels per lane,
# else 64) against 64 everywhere (knob wave_chunk=64), same box: the schedule
# and shard tests on both builds, the headline (4 rounds), 4K and 10k spheres
# (3 rounds), the N = 8 shard (auto = 64, sanity).  usage: bash tools/calls/gpu_r05_call56.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -k "schedule or full_1080 or lead or 10k or image_out" -x -q --timeout 250 --timeout-method thread > $O/t.log 2>&1
step tests $?
timeout -k 10 400 python -u -m pytest tests -m gpu -k "schedule or full_1080 or lead or 10k" -x -q --timeout 250 --timeout-method thread --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/tc.log 2>&1
step tests_checked $?
ROUNDS=4 bash tools/calls/gpu_r05_ab.sh $O/ab cur=product c64=product:wave_chunk=64
step ab $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab4k cur=product c64=product:wave_chunk=64 -- --config rtiow4k --steps 1 --warmup 1
step ab4k $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab10k cur=product c64=product:wave_chunk=64 -- --config spheres10k1080 --steps 2 --warmup 1
step ab10k $?
PROBE_TUNE= timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 > $O/shard8.log 2>&1
step shard8 $?
exit 0
