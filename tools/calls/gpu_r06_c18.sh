# round 6 call 18: counter and executed-work records of the one workload the
# s_setprio rule changed (rtiow4k) and of spheres10k1080 (chunk-level rows).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
CFG=rtiow4k FPL=1 OUT=$O/pmc_4k bash tools/pmc_round.sh > $O/pmc_4k.log 2>&1
step pmc_4k $?
CFG=spheres10k1080 FPL=2 OUT=$O/pmc_10k bash tools/pmc_round.sh > $O/pmc_10k.log 2>&1
step pmc_10k $?
timeout -k 10 400 python -u tools/executed.py $O/executed_raw.json rtiow4k:1 spheres10k1080:2 > $O/executed.log 2>&1
step executed $?
exit 0
