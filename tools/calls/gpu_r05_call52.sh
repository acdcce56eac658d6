# round 5: the N = 8 row shard's tail regions re-swept with end-of-launch
# chunks of 32 (split_probe, shard 7 of 8, 20 frames, 3 passes): the call's
# 1,1,0.25 against 0,1,0.5 / 1,1,0.5 / 2,1,0.25 / 1,0.5,0.25.
# usage: bash tools/calls/gpu_r05_call52.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for pass in 1 2 3; do
  for t in "" "tail=0,1,0.5" "tail=1,1,0.5" "tail=2,1,0.25" "tail=1,0.5,0.25"; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard8.log 2>&1
    step "shard8 $pass $t" $?
  done
done
exit 0
