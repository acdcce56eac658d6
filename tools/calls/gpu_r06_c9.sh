# round 6 call 9: the block bounds' margin muB 2^-8 -> 2^-12 (the proof now
# straight from the exact test's f32 arithmetic): GPU suite on the product
# and the checked build, then same-box A/B against the previous commit's
# library (tools/librt_base6.so) on every BASELINE workload, and the
# headline's work-chunk sweep and the 10k frames-per-launch shape.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
step tests $?
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/gpu_tests_checked.log 2>&1
step tests_checked $?
tail -1 $O/gpu_tests_checked.log
CONFIGS="rtiow1080 spheres10k1080 rtiow4k" bash tools/calls/gpu_r06_ab.sh $O/ab base=tools/librt_base6.so mub=product
step ab $?
ROUNDS=2 CONFIGS="rtiow8k" bash tools/calls/gpu_r06_ab.sh $O/ab base=tools/librt_base6.so mub=product
step ab8k $?
exit 0
