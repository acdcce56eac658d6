# round 6 call 2: drain dumps (per-lane candidate counts) of three workloads
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for w in rtiow1080 spheres10k1080 rtiow4k; do
  timeout -k 10 200 python tools/drain_dump.py $w $O/drain_$w.npy >> $O/drain.log 2>&1
  step $w $?
done
cat $O/drain.log
