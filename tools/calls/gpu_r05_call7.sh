# round 5, call 7: the single-chunk render kernel (no bound-chunk loop) and
# the multi-chunk kernel (chunk-level bounds): headline A/B against the
# round-4 kernel, with and without LDS records; 10k spheres.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product lds9=tools/librt_r05_lds9.so \
    grp=product:item_order=7
step ab $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab10k base=tools/librt_r04_final.so cur=product notop=product:mf_top=0 \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
exit 0
