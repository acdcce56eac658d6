# round 5: the full-size lead-item test on both builds, then the N = 8 row
# shard's block region with lead items (split_probe, shard 7 of 8, 20 frames):
# block_region 16 / 32 / 48 / 64 (the call's) x block_lead 2 (the call's) / 4.
# usage: bash tools/calls/gpu_r05_call42.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lead_items" -x -v --timeout 250 --timeout-method thread > $O/t.log 2>&1
step test $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lead_items" -x -v --timeout 250 --timeout-method thread --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/tc.log 2>&1
step test_checked $?
for pass in 1 2; do
  for t in "" "block_region=48" "block_region=32" "block_region=16" "block_lead=4" "block_lead=4;block_region=48" "block_lead=4;block_region=32" "block_lead=0;block_region=32"; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard8.log 2>&1
    step "shard8 $pass $t" $?
  done
done
exit 0
