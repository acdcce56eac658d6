# round 5: the queue's end-of-launch chunk size (RT_WAVE_CHUNK_TAIL, 16 in the
# product) at 4 / 8 / 32 (compile-time builds of the same sources): the
# headline (3 rounds) and the N = 8 row shard 7 (split_probe, 2 passes).
# usage: bash tools/calls/gpu_r05_call48.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=bevy_raytrace_amd
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab cur=product ct4=$L/librt_hip_ct4.so ct8=$L/librt_hip_ct8.so ct32=$L/librt_hip_ct32.so
step ab $?
for pass in 1 2; do
  for v in "" ct4 ct8 ct32; do
    lib=""; if [ -n "$v" ]; then lib=$L/librt_hip_$v.so; fi
    PROBE_LIB=$lib timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 > $O/shard_${v:-cur}_$pass.log 2>&1
    step "shard $v $pass" $?
  done
done
exit 0
