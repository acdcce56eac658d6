# round-3 GPU call 16: single-row blocks for the row tiling -- N=4 / N=2
# row-block probes, all 8 shards at the driver's form with the new default,
# and the tests that depend on the tiling.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/rowblock_probe.py 4 6 1 > gpurun_out/rowblock_n4.log 2>&1 || exit 161
timeout -k 10 300 python -u tools/rowblock_probe.py 2 8 1 > gpurun_out/rowblock_n2.log 2>&1 || exit 162
timeout -k 10 300 python -u tools/shard_all_probe.py 20 > gpurun_out/shard_all_b1.log 2>&1 || exit 163
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_bench.py -x -v --timeout 150 --timeout-method thread > gpurun_out/t_b1.log 2>&1 || exit 164
