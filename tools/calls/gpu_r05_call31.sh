# round 5, call 31: the pixel region aligned to a frame boundary (knob
# block_align): the schedule-knob identity tests, the headline A/B, and the
# N = 8 / 4 / 2 row shards (tools/split_probe.py).  usage: bash tools/calls/gpu_r05_call31.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "schedule_knobs or item_order" \
    --timeout 200 --timeout-method thread > $O/tests.log 2>&1
step tests $?
bash tools/calls/gpu_r05_ab.sh $O/ab cur=product noalign=product:block_align=0
step ab $?
for pass in 1 2; do
  for t in "" block_align=0; do
    for nk in "8 7" "4 3" "2 1"; do
      PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 $nk 20 >> $O/shards.log 2>&1
      step "shard $nk $pass $t" $?
    done
  done
done
exit 0
