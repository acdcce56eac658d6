# round 5, call 2: the new GPU tests (block bounds at their decision
# boundary, the unculled VALU frames beside the identity tests) and the whole
# intersect suite; the RT_PROFILE build's executed-work counters of every
# workload (tools/executed.py); a ray dump of the headline launch; the PMC
# passes of configs 3-5.  usage: bash tools/calls/gpu_r05_call2.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_intersect.py "tests/test_gpu_parity.py::test_cull_full_1080p64_identical" \
    "tests/test_gpu_configs.py::test_config5_10k_full_frame" > $O/tests.log 2>&1
step tests $?
timeout -k 10 300 python -u tools/executed.py $O/executed_raw.json > $O/executed.log 2>&1
step executed $?
timeout -k 10 120 python -u tools/ray_dump.py $O/ray_dump.npy > $O/ray_dump.log 2>&1
step ray_dump $?
timeout -k 10 200 python -u tools/split_probe.py > $O/split.log 2>&1
step split_probe $?
CFG=spheres10k1080 FPL=2 OUT=$O/pmc_10k bash tools/pmc_round.sh > $O/pmc_10k.log 2>&1
step pmc_10k $?
CFG=rtiow4k FPL=1 OUT=$O/pmc_4k bash tools/pmc_round.sh > $O/pmc_4k.log 2>&1
step pmc_4k $?
CFG=rtiow8k FPL=1 OUT=$O/pmc_8k bash tools/pmc_round.sh > $O/pmc_8k.log 2>&1
step pmc_8k $?
exit 0
