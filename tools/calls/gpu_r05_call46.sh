# round 5: records after the software-pipelined bound-chunk loop: the
# spheres10k1080 PMC passes (two-frame launch), the executed-work counters of
# every workload, then the full record (tools/calls/gpu_r05_record.sh).
# usage: bash tools/calls/gpu_r05_call46.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
CFG=spheres10k1080 FPL=2 OUT=$O/pmc_10k bash tools/pmc_round.sh > $O/pmc_10k.log 2>&1
step pmc_10k $?
cd "$R"
timeout -k 10 400 python -u tools/executed.py $O/executed_raw.json > $O/executed.log 2>&1
step executed $?
bash tools/calls/gpu_r05_record.sh $1/record
step record $?
exit 0
