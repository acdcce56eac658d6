# round 5, call 17: the new schedule-knob identity test; the 8K frame on one
# GPU with the s_setprio rotation on / off (2 rounds each); all 8 N = 8
# shards of the headline (tools/shard_all_probe.py).
# usage: bash tools/calls/gpu_r05_call17.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "schedule_knobs or item_order" \
    --timeout 200 --timeout-method thread > $O/tests.log 2>&1
step tests $?
timeout -k 10 300 python -u tools/shard_all_probe.py 20 8 > $O/shard_all.log 2>&1
step shards $?
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab8k p1=product:prio_mode=1 p0=product:prio_mode=0 \
    -- --config rtiow8k --frames-per-launch 1 --steps 1 --warmup 0
step ab8k $?
exit 0
