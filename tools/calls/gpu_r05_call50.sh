# round 5: RT_WAVE_CHUNK_TAIL 32 / 64 against the product's 16 on the other
# single-GPU workloads: spheres10k1080 (two-frame launches) and rtiow4k (one
# frame), 3 rounds each.  usage: bash tools/calls/gpu_r05_call50.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=bevy_raytrace_amd
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab10k cur=product ct32=$L/librt_hip_ct32.so ct64=$L/librt_hip_ct64.so -- --config spheres10k1080 --steps 2 --warmup 1
step ab10k $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab4k cur=product ct32=$L/librt_hip_ct32.so ct64=$L/librt_hip_ct64.so -- --config rtiow4k --steps 1 --warmup 1
step ab4k $?
exit 0
