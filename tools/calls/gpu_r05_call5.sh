# round 5, call 5: headline A/B after placing the cold walks out of the hot
# loop's way (branch weights): round-4 kernel, product (item order 3 / 7),
# LDS records with queue cap 9; 10k spheres with / without chunk bounds; the
# N=8 shard's collect (image with and without the per-wave release, packed).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product \
    grp=product:item_order=7 lds9=tools/librt_r05_lds9.so
step ab $?
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab10k base=tools/librt_r04_final.so cur=product notop=product:mf_top=0 \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
timeout -k 10 200 python -u tools/split_probe.py 20 8 7 20 10,10 > $O/split.log 2>&1
step split $?
PROBE_TUNE=dsys_release=0 timeout -k 10 200 python -u tools/split_probe.py 20 8 7 20 10,10 >> $O/split.log 2>&1
step split_norel $?
PROBE_PACKED=1 timeout -k 10 200 python -u tools/split_probe.py 20 8 7 20 10,10 >> $O/split.log 2>&1
step split_packed $?
exit 0
