# round-4 GPU call 9: workgroups per CU chosen by the call's size (small
# calls run 1-3 per CU): the GPU suite; the grid probe in auto mode next to
# the fixed settings; the reference's frame through the shim's sequence; the
# other workloads (4K, 10 k spheres, 8K on one GPU) with this build.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04/c9
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 550 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
step tests $?
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > $O/bench_reference1080.json 2> $O/bench_ref.err
step ref $?
timeout -k 10 400 python bench.py --config rtiow4k --steps 1 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 1 --frames-per-launch 1 > $O/bench_4k.json 2> $O/bench_other.err
step bench_4k $?
timeout -k 10 400 python bench.py --config spheres10k1080 --steps 2 --warmup 1 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 2 --frames-per-launch 2 > $O/bench_10k.json 2>> $O/bench_other.err
step bench_10k $?
timeout -k 10 400 python bench.py --config rtiow8k --steps 1 --warmup 0 --no-cpu-baseline \
    --reuse-steps 0 --cull-steps 0 --frames-per-launch 1 > $O/bench_8k_1gpu.json 2>> $O/bench_other.err
step bench_8k_1gpu $?
exit 0
