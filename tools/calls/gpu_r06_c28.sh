# round 6 call 28: the culled line (RT_FLAG_CULL, 12-frame launches) under
# the 128-item chunk + rotation rule (default) against 64-item chunks
# (--tune wave_chunk=64, the round-5 schedule for those launches), interleaved.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for i in 0 1 2 3; do
  timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --reuse-steps 0 > $O/def_$i.json 2> $O/def_$i.err
  step "def $i" $?
  timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --reuse-steps 0 --tune wave_chunk=64 > $O/c64_$i.json 2> $O/c64_$i.err
  step "c64 $i" $?
done
exit 0
