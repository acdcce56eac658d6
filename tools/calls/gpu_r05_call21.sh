# round 5, call 21: the call-shaped tail (1,1,0.25 at about one pixel per
# lane): all 8 N = 8 shards (tools/shard_all_probe.py) and shard 7 against the
# old tail, three passes.  usage: bash tools/calls/gpu_r05_call21.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u tools/shard_all_probe.py 20 8 > $O/shard_all.log 2>&1
step shards $?
for pass in 1 2 3; do
  for t in "" tail=0,1,1; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard8.log 2>&1
    step "shard8 $pass $t" $?
  done
done
exit 0
