# round-4 record of the working kernel plus the other workloads: the default
# bench (with the CPU baseline), the driver-form bench, its rocprofv3 kernel
# trace, the 8 PMC passes of one 20-frame launch (tools/pmc_round.sh), then
# the reference's frame (with the shim sequence), 4K, 10 k spheres and the 8K
# frame on one GPU.  usage: bash tools/calls/gpu_r04_record2.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r04_record.sh $O
step record $?
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
