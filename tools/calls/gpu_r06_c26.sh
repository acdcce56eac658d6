# round 6 call 26: the row shards (N = 8, 4, 2) of the driver's 20-frame
# launch under work chunks of 64 (their rule), 96 and 128 (tools/shard_all_probe.py).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for n in 8 4 2; do
  for c in 64 96 128; do
    PROBE_TUNE="wave_chunk=$c" timeout -k 10 300 python -u tools/shard_all_probe.py 20 $n > $O/shards_n${n}_c$c.log 2>&1
    step "n$n c$c" $?
    grep max $O/shards_n${n}_c$c.log
  done
done
exit 0
