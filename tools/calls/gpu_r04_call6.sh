# round-4 GPU call 6: the reference's frame through the shim's call sequence
# with the collect writing registered host buffers itself; a kernel +
# memory-copy trace of the staged sequence (what carries the D2H copy: an
# SDMA engine or a blit kernel); HBM traffic of the headline launch with and
# without direct output (FETCH_SIZE / WRITE_SIZE, separate passes).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04/c6
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u bench.py --config reference1080 --steps 20 --warmup 4 > $O/bench_reference1080.json 2> $O/bench_ref.err
step bench_ref1080 $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/$O/copytrace" -o run --output-format csv \
    -- python3 "$R/bench.py" --config reference1080 --steps 4 --warmup 1 --no-cpu-baseline --reuse-steps 0 \
    --cull-steps 0 --shim-frames 20 > "$R/$O/copytrace.json" 2> "$R/$O/copytrace.err"
step copytrace $?
C="--steps 20 --warmup 0 --frames-per-launch 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
for d in 1 0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$R/$O/traffic_d${d}_$c" -o run --output-format csv \
        -- python3 "$R/bench.py" $C --tune direct_out=$d > "$R/$O/traffic_d${d}_$c.log" 2>&1
    step "traffic d$d $c" $?
  done
done
exit 0
