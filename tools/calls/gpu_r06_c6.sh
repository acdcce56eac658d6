# round 6 call 6: the tail by the call -- GPU suite (product + checked build),
# same-box A/B against the round-5 kernel (tools/librt_base.so) on every
# BASELINE workload, and the PMC + executed-work records of the two workloads
# whose plan changed (rtiow4k, the 8K frame).  usage: bash tools/calls/gpu_r06_c6.sh <out>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
step tests $?
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/gpu_tests_checked.log 2>&1
step tests_checked $?
tail -1 $O/gpu_tests_checked.log
CONFIGS="rtiow4k rtiow1080 spheres10k1080" bash tools/calls/gpu_r06_ab.sh $O/ab base=tools/librt_base.so tail=product
step ab $?
ROUNDS=2 CONFIGS="rtiow8k" bash tools/calls/gpu_r06_ab.sh $O/ab base=tools/librt_base.so tail=product
step ab8k $?
CFG=rtiow4k FPL=1 OUT=$O/pmc_4k bash tools/pmc_round.sh > $O/pmc_4k.log 2>&1
step pmc_4k $?
CFG=rtiow8k FPL=1 OUT=$O/pmc_8k bash tools/pmc_round.sh > $O/pmc_8k.log 2>&1
step pmc_8k $?
timeout -k 10 400 python -u tools/executed.py $O/executed_raw.json rtiow4k:1 rtiow8k:1 > $O/executed.log 2>&1
step executed $?
exit 0
