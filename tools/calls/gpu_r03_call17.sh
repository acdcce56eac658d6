# round-3 GPU call 17: where a shard launch's extra 6-7 % goes -- per-wave
# start/end/queue-dry times (RT_WAVE_TRACE build) of the full frame and of
# N=8 shards 7 and 0 at the driver's 20-frame launch.
set -o pipefail
mkdir -p gpurun_out
TRACE_CASES="20,1,0;20,8,7;20,8,0" timeout -k 10 300 python -u tools/wave_trace.py > gpurun_out/wave_trace_b1.log 2>&1 || exit 171
