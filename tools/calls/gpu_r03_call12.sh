# round-3 GPU call 12: fused collect + RT_FLAG_IMAGE_OUT -- their parity
# tests, then warm timings (fused off / on, full frame and N=8 shards) and
# the driver-form bench: this build (fused off, on) against the previous
# commit's build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused or image_out or item_order" -x -v --timeout 120 --timeout-method thread > gpurun_out/t_fused.log 2>&1 || exit 121
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 150 --timeout-method thread > gpurun_out/t_bench.log 2>&1 || exit 126
timeout -k 10 300 python -u tools/item_probe.py 20 "" "fused_collect=1" > gpurun_out/fused_probe.log 2>&1 || exit 122
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 > gpurun_out/ab_cur_$i.json 2>/dev/null || exit 123
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --tune fused_collect=1 > gpurun_out/ab_fused_$i.json 2>/dev/null || exit 124
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --lib tools/librt_prev.so > gpurun_out/ab_prev_$i.json 2>/dev/null || exit 125
done
