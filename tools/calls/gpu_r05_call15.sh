# round 5, call 15: s_setprio rotation off (prio_mode 0) against the default
# (1) with the tail knob, at the headline, spheres10k1080, rtiow4k and the
# N = 8 shard (tools/split_probe.py).  usage: bash tools/calls/gpu_r05_call15.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product p0=product:prio_mode=0 \
    p0t05=product:prio_mode=0,tail=0/0.5/1 p0t105=product:prio_mode=0,tail=0/1/0.5 p3=product:prio_mode=3
step ab $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab10k cur=product p0=product:prio_mode=0 \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab4k cur=product p0=product:prio_mode=0 \
    -- --config rtiow4k --frames-per-launch 1 --steps 1 --warmup 1
step ab4k $?
for t in prio_mode=1 prio_mode=0 prio_mode=1 prio_mode=0; do
  PROBE_TUNE=$t timeout -k 10 200 python -u tools/split_probe.py 20 8 7 20 >> $O/shard.log 2>&1
  step "shard $t" $?
done
exit 0
