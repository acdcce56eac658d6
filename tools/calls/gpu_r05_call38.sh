# round 5: lead items (block_lead) at 2 / 3 and 4 with block region 96 against
# the recorded kernel: the headline (5 rounds), 4K (one frame per launch),
# 10k spheres (two-frame launches) and the N = 8 row shard 7 (split_probe),
# plus WRITE_SIZE of l2.  usage: bash tools/calls/gpu_r05_call38.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
REC=rec=bevy_raytrace_amd/librt_hip_rec.so
ROUNDS=5 bash tools/calls/gpu_r05_ab.sh $O/ab $REC l2=product:block_lead=2 l3=product:block_lead=3 l4r96=product:block_lead=4,block_region=96
step ab $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab4k $REC l3=product:block_lead=3 l2=product:block_lead=2 -- --config rtiow4k --steps 1 --warmup 1
step ab4k $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab10k $REC l3=product:block_lead=3 l2=product:block_lead=2 -- --config spheres10k1080 --steps 2 --warmup 1
step ab10k $?
for pass in 1 2; do
  for t in "" block_lead=3 block_lead=2; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard8.log 2>&1
    step "shard8 $pass $t" $?
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$O/pmc_l2" -o run --output-format csv -- \
    python3 $R/bench.py --steps 20 --warmup 0 --frames-per-launch 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --tune block_lead=2 > $O/pmc_l2.log 2>&1
step "pmc l2" $?
exit 0
