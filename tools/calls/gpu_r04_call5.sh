# round-4 GPU call 5: direct output (whole items write their output pixel;
# their frames skip the slots and the collect) and zero-copy host output into
# registered buffers: the GPU suite (product), the new tests once more under
# the bounds-checked build, a same-box A/B against the bitop3 build (driver
# form), and the reference's frame through the shim's call sequence.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04/c5
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step smoke $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "direct or registered or image_out or item_order or tail_split or progressive or multi_pass or checked" \
    -x -v --timeout 200 --timeout-method thread --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/t_checked.log 2>&1
step checked $?
timeout -k 10 550 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
step tests $?
B="--steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
timeout -k 10 120 python -u bench.py $B --lib tools/librt_r04_bitop3.so > $O/ab_warm.json 2>/dev/null
step warm $?
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py $B --lib tools/librt_r04_bitop3.so > $O/ab_base_$i.json 2>/dev/null
  step "base $i" $?
  timeout -k 10 120 python -u bench.py $B > $O/ab_new_$i.json 2>/dev/null
  step "new $i" $?
done
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > $O/bench_reference1080.json 2> $O/bench_ref.err
step bench_ref1080 $?
exit 0
