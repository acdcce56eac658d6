# round-3 first GPU call: op_sel reproduction (tools/isect_diag.py with the
# round-2 build, the op_sel reconstruction, and the op_sel build whose MFMA walk
# is compiled but never taken), the GPU tests on the new build, then the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/isect_diag.py mixed 3 tools/librt_cur_tag.so tools/librt_opsel_tag.so tools/librt_opsel_forcevalu.so > gpurun_out/diag1.log 2>&1 || exit 11
CONCURRENT=1 timeout -k 10 300 python -u tools/isect_diag.py mixed 3 tools/librt_opsel_tag.so > gpurun_out/diag2.log 2>&1 || exit 12
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 13
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 14
