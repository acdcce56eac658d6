# round 5, call 33: shading by walk position (the matrix-core walk's records
# in the walk's order, no permutation load before the shading): the GPU suite
# on the product and the bounds-checked build, then the headline, 10k and 4K
# A/B against the previous library.  usage: bash tools/calls/gpu_r05_call33.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/tests_checked.log 2>&1
step tests_checked $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
step tests $?
bash tools/calls/gpu_r05_ab.sh $O/ab prev=tools/librt_r05_prev.so cur=product
step ab $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab10k prev=tools/librt_r05_prev.so cur=product \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab4k prev=tools/librt_r05_prev.so cur=product \
    -- --config rtiow4k --frames-per-launch 1 --steps 1 --warmup 1
step ab4k $?
exit 0
