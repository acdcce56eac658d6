# round-3 GPU call 20: block-region and tail sweeps with the pixel-major
# order and single-row blocks (warm full / shard 7 / shard 0, F = 20).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/item_probe.py 20 "" "block_region=48" "block_region=64" "block_region=128" "block_region=192" "tail=0,0.5,1" "tail=0,1,0.5" "tail=0,2,1" "tail=1,1,1" "" > gpurun_out/sweep_r3b.log 2>&1 || exit 201
