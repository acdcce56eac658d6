# round-3 GPU call 13: pixel-table entries loaded once per chunk (ctab +
# ds_bpermute): parity tests, then warm timings and the driver-form bench A/B
# against the previous build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "bit_exact or item_order or tail_split or shards or full_1080" -x -v --timeout 150 --timeout-method thread > gpurun_out/t_ctab.log 2>&1 || exit 131
PROBE_LIB=tools/librt_prev.so timeout -k 10 200 python -u tools/item_probe.py 20 "" > gpurun_out/ctab_probe_prev.log 2>&1 || exit 132
timeout -k 10 200 python -u tools/item_probe.py 20 "" > gpurun_out/ctab_probe.log 2>&1 || exit 133
for i in 1 2 3; do
  for lib in bevy_raytrace_amd/librt_hip.so tools/librt_prev.so; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --lib $lib > gpurun_out/ab_$(basename $lib .so)_$i.json 2>/dev/null || exit 134
  done
done
