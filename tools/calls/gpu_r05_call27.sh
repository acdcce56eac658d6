# round 5, call 27: the sphere-parallel threshold (wide_max: the cost model's
# 7 at the headline, against 0 / 2 / 4) at the headline and the N = 8 shard.
# usage: bash tools/calls/gpu_r05_call27.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab cur=product w0=product:wide_max=0 w2=product:wide_max=2 w4=product:wide_max=4
step ab $?
for pass in 1 2; do
  for t in "" wide_max=0 wide_max=2 wide_max=4; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard8.log 2>&1
    step "shard8 $pass $t" $?
  done
done
exit 0
