# round 5, call 19: tail regions for the N = 8 shard (shard 7 of 8,
# tools/split_probe.py, two passes), then the headline and spheres10k1080
# with the shard's best candidates.  usage: bash tools/calls/gpu_r05_call19.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for pass in 1 2; do
  for t in "" tail=1,1,1 tail=2,1,1 tail=1,2,1 tail=1,1,0.5 tail=2,2,1 tail=1,0,1 tail=0.5,1,1 tail=4,1,1; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard.log 2>&1
    step "shard $pass $t" $?
  done
done
bash tools/calls/gpu_r05_ab.sh $O/ab cur=product t111=product:tail=1/1/1 t211=product:tail=2/1/1 t051=product:tail=0/0.5/1
step ab $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab10k cur=product t111=product:tail=1/1/1 t211=product:tail=2/1/1 \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
exit 0
