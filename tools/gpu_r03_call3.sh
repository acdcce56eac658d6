# round-3 GPU call 3: op_sel variants on the current tree (tools/opsel_variants.py),
# the GPU tests (incl. the side-by-side walk tests), the driver-form bench, the
# reference's own frame through the shim's call sequence, the two-stream
# launch split probe and the phase profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/isect_diag.py mixed 3 tools/librt_cur_tag.so tools/librt_opsel_fixed.so tools/librt_opsel_owned.so > gpurun_out/diag3.log 2>&1 || exit 31
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 32
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 33
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > gpurun_out/bench_reference1080.json 2> gpurun_out/bench_reference1080.err || exit 34
timeout -k 10 300 python -u tools/shard_split_probe.py 20 2 > gpurun_out/shard_split.log 2>&1 || exit 35
timeout -k 10 300 python -u tools/prof_phases.py 20,1,0 20,8,7 20,8,0 > gpurun_out/phases.log 2>&1 || exit 36
