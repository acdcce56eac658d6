# Same-box A/B of the round's kernel against the round-3 kernel (+ the
# in-kernel clock sums, tools/librt_r04_base.so): the headline driver form 3+3
# interleaved, then 10,000 spheres 1+1.  usage: bash tools/calls/gpu_r04_round_ab.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r04_sens.sh $O tools/librt_r04_base.so
step headline $?
B="--config spheres10k1080 --steps 2 --warmup 1 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --frames-per-launch 2"
timeout -k 10 300 python bench.py $B > $O/k10_new.json 2>/dev/null
step k10_new $?
timeout -k 10 300 python bench.py $B --lib tools/librt_r04_base.so > $O/k10_r3.json 2>/dev/null
step k10_r3 $?
exit 0
