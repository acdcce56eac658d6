# round 6 call 1: the new GPU tests (cross-rank check, MFMA accumulation),
# smoke, one driver-form bench line.  usage: bash tools/calls/gpu_r06_c1.sh <out>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
RT_MFMA_ACC_REPORT=$O/mfma_acc.json timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma_acc.py tests/test_gpu_bench.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1
step tests $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step smoke $?
timeout -k 10 300 python bench.py --steps 20 --warmup 4 > $O/bench.json 2> $O/bench.err
step bench $?
cat $O/bench.json | head -c 600
exit 0
