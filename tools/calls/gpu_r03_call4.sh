# round-3 GPU call 4: op_sel ubench against a scalar fma reference, GPU tests,
# reference1080 with registered host buffers, drain A/B (nested / flat / flat
# + next-record prefetch) at the driver's 20-frame launch, the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 ./tools/ubench/opsel_mfma 2 > gpurun_out/opsel_mfma3.log 2>&1 || exit 40
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 41
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > gpurun_out/bench_reference1080.json 2> gpurun_out/bench_reference1080.err || exit 42
for i in 1 2; do
  for lib in bevy_raytrace_amd/librt_hip.so tools/librt_flat.so tools/librt_flatpf.so; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --lib $lib > gpurun_out/ab_$(basename $lib .so)_$i.json 2>/dev/null || exit 43
  done
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 45
timeout -k 10 400 python -u tools/launch_cost_probe.py "" "RT_TAIL=0,0,0" "RT_BLOCK_REGION=192" > gpurun_out/launch_cost.log 2>&1 || exit 46
