# round 5, call 11: block region default 64 against 96 / 80 / 56 (headline,
# driver form), the N = 8 shard at 96 / 64 / 56 (tools/split_probe.py), then
# the per-workload counter record of the product (tools/calls/gpu_r05_pmc.sh).
# usage: bash tools/calls/gpu_r05_call11.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product b96=product:block_region=96 \
    b80=product:block_region=80 b56=product:block_region=56
step ab $?
for br in 96 64 56; do
  PROBE_TUNE=block_region=$br timeout -k 10 200 python -u tools/split_probe.py 20 8 7 20 >> $O/shard.log 2>&1
  step "shard $br" $?
done
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab10k base=tools/librt_r04_final.so cur=product b96=product:block_region=96 \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
bash tools/calls/gpu_r05_pmc.sh $O/pmc
step pmc $?
exit 0
