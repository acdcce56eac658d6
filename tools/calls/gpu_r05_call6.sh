# round 5, call 6: bisect the headline's +2.3 % against the round-4 kernel
# (grouped-order code / chunk-bound code compiled out) and the 10k no-chunk
# path's +13 % (the chunk loads as hipcc strength-reduces them).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product \
    nogrp=tools/librt_r05_nogrp.so notopc=tools/librt_r05_notopc.so neither=tools/librt_r05_neither.so \
    lsr=tools/librt_r05_lsr.so
step ab $?
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab10k base=tools/librt_r04_final.so cur=product \
    notop=product:mf_top=0 lsr_notop=tools/librt_r05_lsr.so:mf_top=0 neither=tools/librt_r05_neither.so \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
exit 0
