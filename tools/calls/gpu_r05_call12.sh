# round 5, call 12: the block region by the call (16 spp / D in [64, 128])
# against fixed regions: headline, spheres10k1080 (two-frame launches),
# rtiow4k and the 8K frame on one GPU.  usage: bash tools/calls/gpu_r05_call12.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product b96=product:block_region=96
step ab $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab10k base=tools/librt_r04_final.so cur=product b96=product:block_region=96 \
    b160=product:block_region=160 -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab4k base=tools/librt_r04_final.so cur=product b96=product:block_region=96 \
    -- --config rtiow4k --frames-per-launch 1 --steps 1 --warmup 1
step ab4k $?
ROUNDS=1 bash tools/calls/gpu_r05_ab.sh $O/ab8k cur=product b96=product:block_region=96 \
    -- --config rtiow8k --frames-per-launch 1 --steps 1 --warmup 0
step ab8k $?
exit 0
