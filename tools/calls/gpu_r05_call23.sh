# round 5, call 23: the 16 x 16 matrix-core walk (-DRT_MF16 builds,
# tools/librt_r05_mf16*.so): the GPU suite on its bounds-checked build, then
# on its product build, then the headline A/B against the product and the
# round-4 library.  usage: bash tools/calls/gpu_r05_call23.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
DS="--deselect tests/test_gpu_parity.py::test_native_library_is_in_tree"
timeout -k 10 400 python -u -m pytest tests/test_gpu_intersect.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 200 --timeout-method thread --rt-lib tools/librt_r05_mf16_checked.so $DS > $O/tests_checked_quick.log 2>&1
step tests_checked_quick $?
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    --rt-lib tools/librt_r05_mf16.so $DS > $O/tests_mf16.log 2>&1
step tests_mf16 $?
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product mf16=tools/librt_r05_mf16.so
step ab $?
exit 0
