# round 6 call 24: the s_setprio rotation with the 128-item chunks (the
# multi-frame whole-frame launches): GPU suite, then same-box A/B at the
# headline (6 rounds) and the bench's default 24-frame shape (3 rounds)
# against the previous commit's library.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
step tests $?
tail -1 $O/gpu_tests.log
ROUNDS=6 CONFIGS="rtiow1080" bash tools/calls/gpu_r06_ab.sh $O/ab base=tools/librt_base11.so prio=product
step ab $?
for i in 1 2 3; do
  for a in base prio; do
    L=""; [ $a = base ] && L="--lib tools/librt_base11.so"
    timeout -k 10 200 python -u bench.py --steps 24 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 $L > $O/d24_${a}_$i.json 2>/dev/null
    step "d24 $a $i" $?
  done
done
exit 0
