# round-3 GPU call 23: the widened full-size parity samples (1080p/64 on 70
# rows, 4K on 24, all 8 config-4 shards, config 5 on 12 rows), timed.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/t_wide.log 2>&1 || exit 231
