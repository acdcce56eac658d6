# round 5, call 8: the product with the single-chunk LDS-record kernel and
# the multi-chunk kernel: the GPU suite on it and on the checked build, the
# headline A/B against the round-4 kernel, 10k spheres, the N=8 shard's
# launch with the block region sized down (split probe).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/gpu_tests_checked.log 2>&1
step tests_checked $?
bash tools/calls/gpu_r05_ab.sh $O/ab --tests base=tools/librt_r04_final.so cur=product
step ab $?
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab10k base=tools/librt_r04_final.so cur=product \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
for br in 96 48 24 12; do
  PROBE_TUNE=block_region=$br timeout -k 10 200 python -u tools/split_probe.py 20 8 7 20 >> $O/split.log 2>&1
  step "split br $br" $?
done
exit 0
