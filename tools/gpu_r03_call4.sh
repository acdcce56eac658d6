# round-3 GPU call 4: op_sel ubench against a scalar fma reference, GPU tests,
# reference1080 with registered host buffers, flat-drain A/B at the driver's
# 20-frame launch, the driver-form bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 ./tools/ubench/opsel_mfma 2 > gpurun_out/opsel_mfma3.log 2>&1 || exit 40
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 41
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > gpurun_out/bench_reference1080.json 2> gpurun_out/bench_reference1080.err || exit 42
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 > gpurun_out/ab_prod_$i.json 2>/dev/null || exit 43
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --lib tools/librt_flat.so > gpurun_out/ab_flat_$i.json 2>/dev/null || exit 44
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 45
