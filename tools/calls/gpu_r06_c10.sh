# round 6 call 10: the final kernel's counter records (PMC passes of one
# bench-shaped launch per BASELINE workload, tools/pmc_round.sh) and executed-
# work records (RT_PROFILE build, tools/executed.py), then the measurement
# record (tools/calls/gpu_r06_record.sh) -- the bench lines carry the records
# committed before them, so this call's record lines are re-run after the
# counters are summarised (call 11).  usage: bash tools/calls/gpu_r06_c10.sh <out>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
CFG=rtiow1080 FPL=20 OUT=$O/pmc_1080 bash tools/pmc_round.sh > $O/pmc_1080.log 2>&1
step pmc_1080 $?
CFG=spheres10k1080 FPL=2 OUT=$O/pmc_10k bash tools/pmc_round.sh > $O/pmc_10k.log 2>&1
step pmc_10k $?
CFG=rtiow4k FPL=1 OUT=$O/pmc_4k bash tools/pmc_round.sh > $O/pmc_4k.log 2>&1
step pmc_4k $?
CFG=rtiow8k FPL=1 OUT=$O/pmc_8k bash tools/pmc_round.sh > $O/pmc_8k.log 2>&1
step pmc_8k $?
timeout -k 10 500 python -u tools/executed.py $O/executed_raw.json > $O/executed.log 2>&1
step executed $?
exit 0
