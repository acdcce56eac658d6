# round-3 GPU call 19: is the shard's extra wait the slot stores? Warm
# full / shard 7 / shard 0 times (F = 20) of the product build, of the
# product with all block items (block_region huge), and of a diagnostic build
# without the slot stores.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/item_probe.py 20 "" "block_region=100000" > gpurun_out/diag_store_a.log 2>&1 || exit 191
PROBE_LIB=tools/librt_nostore.so timeout -k 10 300 python -u tools/item_probe.py 20 "" > gpurun_out/diag_store_b.log 2>&1 || exit 192
