# round-3 GPU call 6: A/B at the driver's 20-frame launch of item starts with
# kernarg fields read as values (startv) and of the balanced drain (bal, on
# top of startv); the GPU tests with the balanced-drain build in place of the
# shipped library (this box's copy only); launch-cost fit of cur vs startv.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for lib in bevy_raytrace_amd/librt_hip.so tools/librt_startv.so tools/librt_bal.so; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --lib $lib > gpurun_out/ab_$(basename $lib .so)_$i.json 2>/dev/null || exit 60
  done
done
cp tools/librt_bal.so bevy_raytrace_amd/librt_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_bal.log 2>&1 || exit 61
PROBE_LIB=tools/librt_startv.so PROBE_F=10,40 timeout -k 10 300 python -u tools/launch_cost_probe.py "" > gpurun_out/launch_cost_startv.log 2>&1 || exit 62
PROBE_LIB=tools/librt_bal.so PROBE_F=10,40 timeout -k 10 300 python -u tools/launch_cost_probe.py "" > gpurun_out/launch_cost_bal.log 2>&1 || exit 63
