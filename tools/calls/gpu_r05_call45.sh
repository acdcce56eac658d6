# round 5: the matrix-core walk of longer lists as one block pipeline across
# its walk chunks (rt_render_multi_kernel) against the previous commit's
# library: the 10k-sphere workload (two-frame launches, 4 rounds) and its
# identity tests.  usage: bash tools/calls/gpu_r05_call45.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -k "10k or 10000 or multi or chunk or intersect" -x -q --timeout 250 --timeout-method thread > $O/t.log 2>&1
step tests $?
ROUNDS=4 bash tools/calls/gpu_r05_ab.sh $O/ab10k prev=bevy_raytrace_amd/librt_hip_prev2.so cur=product -- --config spheres10k1080 --steps 2 --warmup 1
step ab10k $?
exit 0
