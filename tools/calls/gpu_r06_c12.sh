# round 6 call 12: the forward rows' margins (L' = (1 + 2^-12) L + 2^-8 |C|_1
# + 2^-14, c0 = fma(2^-9, |o|_1, -k1); were (1 + 2^-3) L + 2^-7 |C|_1 and
# 2^-7): GPU suite on the product and the checked build, then same-box A/B
# against the previous commit's library (tools/librt_base7.so) on every
# BASELINE workload; arm fwdr2 adds the bound radius R^2 = (1 + 2^-5 + 2^-10) L^2 (was 1 + 2^-4).
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
CONFIGS="rtiow1080 spheres10k1080 rtiow4k" bash tools/calls/gpu_r06_ab.sh $O/ab base=tools/librt_base7.so fwd=tools/librt_fwd.so fwdr2=product
step ab $?
ROUNDS=2 CONFIGS="rtiow8k" bash tools/calls/gpu_r06_ab.sh $O/ab base=tools/librt_base7.so fwd=tools/librt_fwd.so fwdr2=product
step ab8k $?
exit 0
