# round-3 GPU call 25: slot stores through a per-wave LDS buffer -- parity (render
# tests, smoke), then A/B warm full / shard
# times (F = 20) against the previous commit's build, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_sb.log 2>&1 || exit 251
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_sb.log 2>&1 || exit 252
for i in 1 2; do
  PROBE_LIB=tools/librt_base.so timeout -k 10 200 python -u tools/item_probe.py 20 "" > gpurun_out/ab_sb_base_$i.log 2>&1 || exit 253
  timeout -k 10 200 python -u tools/item_probe.py 20 "" > gpurun_out/ab_sb_new_$i.log 2>&1 || exit 254
done
