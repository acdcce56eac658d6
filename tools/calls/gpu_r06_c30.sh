# round 6 call 30: knobs on the N = 8 row shards of the driver's 20-frame
# launch (tools/shard_all_probe.py): lead items of 3 / 4 / 6 blocks against
# the call's 2, block region 48 / 80 against 64 (c27 swept them on the headline).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
i=0
for t in "" "block_lead=3" "block_lead=4" "block_lead=6" "block_region=48" "block_region=80" ""; do
  PROBE_TUNE="$t" timeout -k 10 300 python -u tools/shard_all_probe.py 20 8 > $O/n8_${i}.log 2>&1
  step "n8 [$t]" $?
  echo "[$t] $(grep 'bench-like' $O/n8_${i}.log | tail -1)"
  i=$((i+1))
done
exit 0
