# round 5: the bound-chunk loop software-pipelined (the next chunk's rows load
# while this chunk's ORs run; rt_render_multi_kernel only): the 10k-sphere
# workload (two-frame launches, 4 rounds) and the headline (3 rounds) against
# the previous commit's library, then the 10k identity tests on both builds.
# usage: bash tools/calls/gpu_r05_call44.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -k "10k or 10000 or multi or chunk" -x -q --timeout 250 --timeout-method thread > $O/t.log 2>&1
step tests $?
ROUNDS=4 bash tools/calls/gpu_r05_ab.sh $O/ab10k prev=bevy_raytrace_amd/librt_hip_prev.so cur=product -- --config spheres10k1080 --steps 2 --warmup 1
step ab10k $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab prev=bevy_raytrace_amd/librt_hip_prev.so cur=product
step ab $?
timeout -k 10 400 python -u -m pytest tests -m gpu -k "10k or 10000 or multi or chunk" -x -q --timeout 250 --timeout-method thread --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/tc.log 2>&1
step tests_checked $?
exit 0
