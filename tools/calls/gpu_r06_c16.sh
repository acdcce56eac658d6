# round 6 call 16: chunk-level bound rows with their own split of the proof's
# slack (R^2 = (1 + 2^-7 + 2^-9) L^2, 4 muB): GPU suite on the product and
# the checked build, same-box A/B on the 10,000-sphere list (the only
# BASELINE workload with chunk-level rows) against the previous commit's
# library; then the one-frame 4K launch's slow runs: 6 rounds of the product,
# the s_setprio rotation on, and the tail on.
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
ROUNDS=5 CONFIGS="spheres10k1080" bash tools/calls/gpu_r06_ab.sh $O/ab base=tools/librt_base8.so chunk=product
step ab $?
ROUNDS=6 CONFIGS="rtiow4k" bash tools/calls/gpu_r06_ab.sh $O/ab4k prod=product prio1=product:prio_mode=1 tail1=product:tail_split=1
step ab4k $?
exit 0
