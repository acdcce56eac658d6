# round-4 multi-rank rehearsal of the committed kernel on one GPU: all 8 N=8
# shards at the driver's 20-frame launch (tools/shard_all_probe.py: the
# render-only speedup prediction), then 8 ranks through the IPC image path
# (gloo control, every rank writing its rows into rank 0's mapped image with
# system-scope stores + release, rank 0 acquiring) and 2 ranks through the
# RCCL gather path, frames checksummed against N=1.
# usage: bash tools/calls/gpu_r04_multi.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u tools/shard_all_probe.py 20 8 > $O/shard_all.log 2>&1
step shards $?
A="--steps 2 --warmup 1 --frames-per-launch 2 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --check"
timeout -k 10 200 python -u bench.py --config config1 $A > $O/n1_c1.json 2> $O/n.err
step n1_c1 $?
timeout -k 10 300 python -u bench.py --config config1 $A --gpus 8 --same-device --dist-backend gloo --gather ipc > $O/n8_c1.json 2>> $O/n.err
step n8_c1 $?
timeout -k 10 200 python -u bench.py $A > $O/n1_1080.json 2>> $O/n.err
step n1_1080 $?
timeout -k 10 300 python -u bench.py $A --gpus 8 --same-device --dist-backend gloo --gather ipc > $O/n8_1080.json 2>> $O/n.err
step n8_1080 $?
timeout -k 10 300 python -u bench.py $A --gpus 2 --same-device --dist-backend gloo --gather rccl > $O/n2_rccl_1080.json 2>> $O/n.err
step n2_rccl $?
exit 0
