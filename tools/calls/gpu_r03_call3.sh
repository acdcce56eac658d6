# round-3 GPU call 3: op_sel isolation ubench (partner-wave modes), the GPU
# tests, the driver-form bench, the reference's own frame through the shim's
# call sequence, the flat-drain A/B, phase profiles, the two-stream launch
# split and the N=8 row-block probes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 ./tools/ubench/opsel_mfma 2 > gpurun_out/opsel_mfma2.log 2>&1 || exit 30
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 32
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 33
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > gpurun_out/bench_reference1080.json 2> gpurun_out/bench_reference1080.err || exit 34
timeout -k 10 300 python -u tools/ab.py bevy_raytrace_amd/librt_hip.so tools/librt_flat.so --reps 6 > gpurun_out/ab_flat.log 2>&1 || exit 35
RT_PROF_LIB=tools/librt_hip_prof.so timeout -k 10 300 python -u tools/prof_phases.py 20,1,0 20,8,7 > gpurun_out/phases.log 2>&1 || exit 36
RT_PROF_LIB=tools/librt_hip_prof_flat.so timeout -k 10 300 python -u tools/prof_phases.py 20,1,0 20,8,7 > gpurun_out/phases_flat.log 2>&1 || exit 37
timeout -k 10 300 python -u tools/shard_split_probe.py 20 2 > gpurun_out/shard_split.log 2>&1 || exit 38
timeout -k 10 300 python -u tools/rowblock_probe.py 8 5 8 9 > gpurun_out/rowblock.log 2>&1 || exit 39
