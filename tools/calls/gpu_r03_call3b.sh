# round-3 GPU call 3b: the reference's own frame through the shim's call
# sequence, the two-stream launch split probe and the phase profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > gpurun_out/bench_reference1080.json 2> gpurun_out/bench_reference1080.err || exit 34
timeout -k 10 300 python -u tools/shard_split_probe.py 20 2 > gpurun_out/shard_split.log 2>&1 || exit 35
timeout -k 10 300 python -u tools/prof_phases.py 20,1,0 20,8,7 20,8,0 > gpurun_out/phases.log 2>&1 || exit 36
