# round-3 GPU call 29: the other workloads with the shipped kernel (4K/256/32,
# 10 k spheres, the 8K/1024 frame on one GPU, the reference's own 1080p/1 spp
# frame through the shim's call sequence) and smoke.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
step smoke $?
timeout -k 10 400 python bench.py --config rtiow4k --steps 1 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 1 --frames-per-launch 1 > gpurun_out/bench_4k.json 2> gpurun_out/bench_other.err
step bench_4k $?
timeout -k 10 400 python bench.py --config spheres10k1080 --steps 2 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 2 --frames-per-launch 2 > gpurun_out/bench_10k.json 2>> gpurun_out/bench_other.err
step bench_10k $?
timeout -k 10 400 python bench.py --config rtiow8k --steps 1 --warmup 0 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 0 --frames-per-launch 1 > gpurun_out/bench_8k_1gpu.json 2>> gpurun_out/bench_other.err
step bench_8k_1gpu $?
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > gpurun_out/bench_reference1080.json 2>> gpurun_out/bench_other.err
step bench_ref1080 $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
