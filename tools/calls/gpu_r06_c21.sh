# round 6 call 21: the headline's counter and executed-work records after the
# work-chunk rule (the only workload it changes).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
CFG=rtiow1080 FPL=20 OUT=$O/pmc_1080 bash tools/pmc_round.sh > $O/pmc_1080.log 2>&1
step pmc_1080 $?
timeout -k 10 400 python -u tools/executed.py $O/executed_raw.json rtiow1080:20 > $O/executed.log 2>&1
step executed $?
exit 0
