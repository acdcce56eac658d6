# round 6 call 29: the N = 8 / 4 row shards of the driver's 20-frame launch
# under work chunks below the rule's 64 (32, 48) against 64
# (tools/shard_all_probe.py; c26 covered 64 / 96 / 128).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for n in 8 4; do
  for c in 64 32 48 64; do
    PROBE_TUNE="wave_chunk=$c" timeout -k 10 300 python -u tools/shard_all_probe.py 20 $n > $O/shards_n${n}_c${c}_$RANDOM.log 2>&1
    step "n$n c$c" $?
  done
done
grep -H max $O/*.log
exit 0
