# round-3 GPU call 5: the flat-drain product through the GPU tests, wave traces
# of the N=8 shard and the full frame (where the per-launch fixed cost goes),
# phase profile, the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 51
TRACE_CASES="5,8,7;20,8,7;20,1,0" timeout -k 10 300 python -u tools/wave_trace.py > gpurun_out/wave_trace.log 2>&1 || exit 52
RT_PROF_LIB=tools/librt_hip_prof.so timeout -k 10 300 python -u tools/prof_phases.py 20,1,0 20,8,7 > gpurun_out/phases.log 2>&1 || exit 53
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 54
