# round 6 call 32: the scheduler options of the render kernels' compile
# (-mllvm -amdgpu-use-amdgpu-trackers = trk; + -amdgpu-sched-strategy=max-ilp
# = combo; max-ilp alone) against the product build: headline (4 rounds),
# 4K and 10k spheres (3 rounds), the N = 8 row shards.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=4 CONFIGS="rtiow1080" bash tools/calls/gpu_r06_ab.sh $O base=product trk=tools/librt_sched_trk.so maxilp=tools/librt_sched_maxilp.so combo=tools/librt_sched_combo.so
step h $?
ROUNDS=3 CONFIGS="rtiow4k spheres10k1080" bash tools/calls/gpu_r06_ab.sh $O base=product trk=tools/librt_sched_trk.so combo=tools/librt_sched_combo.so
step o $?
for l in product trk combo product; do
  L=""; [ $l != product ] && L=tools/librt_sched_$l.so
  PROBE_LIB=$L timeout -k 10 300 python -u tools/shard_all_probe.py 20 8 > $O/shards_${l}_$RANDOM.log 2>&1
  step "shards $l" $?
done
grep -H "bench-like" $O/shards_*.log
exit 0
