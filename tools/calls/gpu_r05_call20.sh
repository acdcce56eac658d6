# round 5, call 20: tail regions for the N = 8 / 4 / 2 row shards of the
# headline (the last shard of each, tools/split_probe.py, two passes).
# usage: bash tools/calls/gpu_r05_call20.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for pass in 1 2; do
  for t in "" tail=1,1,0.5 tail=1,1,0.25 tail=1.5,1,0.5 tail=1,0.5,0.5 tail=0.5,1,0.5; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard8.log 2>&1
    step "shard8 $pass $t" $?
  done
  for t in "" tail=1,1,0.5 tail=0.5,1,0.5; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 4 3 20 >> $O/shard4.log 2>&1
    step "shard4 $pass $t" $?
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 2 1 20 >> $O/shard2.log 2>&1
    step "shard2 $pass $t" $?
  done
done
exit 0
