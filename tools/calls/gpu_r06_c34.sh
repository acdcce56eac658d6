# round 6 call 34: the build with the AMDGPU scheduler trackers -- the GPU
# suite, then the counter records (PMC passes, tools/pmc_round.sh) and the
# executed-work records (RT_PROFILE build) the bench lines carry.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
step tests $?
tail -1 $O/gpu_tests.log
CFG=rtiow1080 FPL=20 OUT=$O/pmc_1080 bash tools/pmc_round.sh > $O/pmc_1080.log 2>&1
step pmc_1080 $?
CFG=rtiow4k FPL=1 OUT=$O/pmc_4k bash tools/pmc_round.sh > $O/pmc_4k.log 2>&1
step pmc_4k $?
CFG=spheres10k1080 FPL=2 OUT=$O/pmc_10k bash tools/pmc_round.sh > $O/pmc_10k.log 2>&1
step pmc_10k $?
CFG=rtiow8k FPL=1 OUT=$O/pmc_8k bash tools/pmc_round.sh > $O/pmc_8k.log 2>&1
step pmc_8k $?
timeout -k 10 400 python -u tools/executed.py $O/executed_raw.json > $O/executed.log 2>&1
step executed $?
exit 0
