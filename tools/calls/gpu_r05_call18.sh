# round 5, call 18: the N = 8 shard's 20-frame launch (shard 7 of 8,
# tools/split_probe.py) over tail / block-region / grid / priority knobs,
# two interleaved passes.  usage: bash tools/calls/gpu_r05_call18.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for pass in 1 2; do
  for t in "" tail=0,2,2 tail=0,0.5,1 tail=0,1,2 tail=0,2,1 tail=1,1,1 block_region=96 block_region=128 \
           prio_mode=3 wg_per_cu=3 tail=0,0,2; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard.log 2>&1
    step "shard $pass $t" $?
  done
done
exit 0
