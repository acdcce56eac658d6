# round-3 GPU call 10: pixel-major item order (item_order=3, the new default)
# through the whole GPU suite, then the driver-form bench A/B against the
# previous commit's build, then the N=8 shard timing (all 8 shards, warm and
# after a 1 ms idle gap) with the new order.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 101
for i in 1 2 3; do
  for lib in bevy_raytrace_amd/librt_hip.so tools/librt_prev.so; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --lib $lib > gpurun_out/ab_$(basename $lib .so)_$i.json 2> gpurun_out/ab_$(basename $lib .so)_$i.err || exit 102
  done
done
timeout -k 10 300 python -u tools/shard_all_probe.py 20 > gpurun_out/shard_all.log 2>&1 || exit 103
