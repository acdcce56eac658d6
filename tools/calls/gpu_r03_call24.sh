# round-3 GPU call 24: item starts reuse the held pixel-table entry when the
# pixel repeats -- parity (render tests, smoke), then A/B warm full / shard
# times (F = 20) against the previous commit's build, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_pk.log 2>&1 || exit 241
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_pk.log 2>&1 || exit 242
for i in 1 2; do
  PROBE_LIB=tools/librt_base.so timeout -k 10 200 python -u tools/item_probe.py 20 "" > gpurun_out/ab_pk_base_$i.log 2>&1 || exit 243
  timeout -k 10 200 python -u tools/item_probe.py 20 "" > gpurun_out/ab_pk_new_$i.log 2>&1 || exit 244
done
