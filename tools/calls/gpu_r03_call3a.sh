# round-3 GPU call 3a: op_sel isolation ubench (partner-wave modes), the GPU tests, the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 ./tools/ubench/opsel_mfma 2 > gpurun_out/opsel_mfma2.log 2>&1 || exit 30
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 32
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 33
