# round-4 GPU call 1: smoke; the GPU suite once against the bounds-checked
# build (librt_hip_checked.so: every computed index of the kernels checked,
# VERDICT r03 next-1), then against the product build; the default bench.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.log 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    --rt-lib bevy_raytrace_amd/librt_hip_checked.so > gpurun_out/r04/gpu_tests_checked.log 2>&1 || exit 12
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r04/gpu_tests.log 2>&1 || exit 13
timeout -k 10 300 python -u bench.py > gpurun_out/r04/bench_default.json 2> gpurun_out/r04/bench_default.err || exit 14
