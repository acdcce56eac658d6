# round-4 GPU call 7: the cleaned-up direct output (device-local outputs only)
# through the GPU suite; the reference's frame through the shim's sequence
# with 4 (default), 3 and 2 render workgroups per CU (a CU slot left free for
# the runtime's D2H blit kernel, which cannot start beside a full persistent
# render: the copy trace of call 6).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04/c7
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 550 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
step tests $?
for w in 3 2; do
  timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 --no-cpu-baseline \
      --reuse-steps 0 --cull-steps 0 --tune wg_per_cu=$w > $O/ref1080_wg$w.json 2> $O/ref1080_wg$w.err
  step "ref wg$w" $?
done
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > $O/bench_reference1080.json 2> $O/bench_ref.err
step ref $?
exit 0
