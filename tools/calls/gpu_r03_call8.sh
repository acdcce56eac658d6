# round-3 GPU call 8: the perm-encoded candidate queue (sgn_bytes, spread
# group index, per-lane write pointer) through the whole GPU suite, then an
# A/B against the previous commit's build (tools/librt_prev.so) at the
# driver's 20-frame launch, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 81
for i in 1 2 3; do
  for lib in bevy_raytrace_amd/librt_hip.so tools/librt_prev.so; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --lib $lib > gpurun_out/ab_$(basename $lib .so)_$i.json 2> gpurun_out/ab_$(basename $lib .so)_$i.err || exit 82
  done
done
