# round-3 GPU call 30: bench.py with no flags (the default N=1 run), timed.
set -o pipefail
mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 301
echo "wall $(( $(date +%s) - start )) s"
