# round-5 counter record after the call-sized priority rule (the headline,
# rtiow4k and the 8K frame changed; spheres10k1080 keeps call 13's record):
# the PMC passes of one bench-shaped launch each (tools/pmc_round.sh:
# rtiow1080 20 frames, spheres10k1080 2, rtiow4k 1, the 8K frame on one GPU)
# and the RT_PROFILE build's executed-work counters (tools/executed.py).
# tools/pmc_summary.py / tools/executed_summary.py turn them into
# profiles/pmc_traffic.json / profiles/executed.json, which the bench lines of
# tools/calls/gpu_r05_record.sh then carry.  usage: bash tools/calls/gpu_r05_pmc.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
CFG=rtiow1080 FPL=20 OUT=$O/pmc_1080 bash tools/pmc_round.sh > $O/pmc_1080.log 2>&1
step pmc_1080 $?


CFG=rtiow4k FPL=1 OUT=$O/pmc_4k bash tools/pmc_round.sh > $O/pmc_4k.log 2>&1
step pmc_4k $?
CFG=rtiow8k FPL=1 OUT=$O/pmc_8k bash tools/pmc_round.sh > $O/pmc_8k.log 2>&1
step pmc_8k $?
timeout -k 10 400 python -u tools/executed.py $O/executed_raw.json > $O/executed.log 2>&1
step executed $?
exit 0
