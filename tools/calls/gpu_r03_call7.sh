# round-3 GPU call 7: the balanced-drain build (tools/librt_bal.so) through
# the intersection parity tests first (stderr kept), then the whole GPU suite,
# then an A/B against the shipped build at the driver's 20-frame launch.
set -o pipefail
mkdir -p gpurun_out
cp bevy_raytrace_amd/librt_hip.so /tmp/librt_hip_shipped.so
cp tools/librt_bal.so bevy_raytrace_amd/librt_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_intersect.py -x -v --timeout 120 --timeout-method thread > gpurun_out/bal_isect.log 2>&1 || exit 70
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_bal.log 2>&1 || exit 71
cp /tmp/librt_hip_shipped.so bevy_raytrace_amd/librt_hip.so
for i in 1 2; do
  for lib in bevy_raytrace_amd/librt_hip.so tools/librt_bal.so; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --lib $lib > gpurun_out/ab_$(basename $lib .so)_$i.json 2> gpurun_out/ab_$(basename $lib .so)_$i.err || exit 72
  done
done
