# round 5: the counter record of rtiow4k, the 8K frame and spheres10k1080
# again after the block region became the call's (tools/calls/gpu_r05_pmc.sh's
# passes and the executed-work counters; the headline's record is call 11's,
# same block region).  usage: bash tools/calls/gpu_r05_pmc2.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
CFG=spheres10k1080 FPL=2 OUT=$O/pmc_10k bash tools/pmc_round.sh > $O/pmc_10k.log 2>&1
step pmc_10k $?
CFG=rtiow4k FPL=1 OUT=$O/pmc_4k bash tools/pmc_round.sh > $O/pmc_4k.log 2>&1
step pmc_4k $?
CFG=rtiow8k FPL=1 OUT=$O/pmc_8k bash tools/pmc_round.sh > $O/pmc_8k.log 2>&1
step pmc_8k $?
timeout -k 10 400 python -u tools/executed.py $O/executed_raw.json > $O/executed.log 2>&1
step executed $?
exit 0
