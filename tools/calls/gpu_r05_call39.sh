# round 5: lead items by the call (m = 2 where a pixel region exists) against
# the recorded kernel: the schedule-knob identity and 1080p tests on both
# builds, the headline A/B (5 rounds, with lead 4 + block region 96 beside),
# and the N = 2 / 4 / 8 row shards (their last shard, split_probe) with the
# call's lead items and without.  usage: bash tools/calls/gpu_r05_call39.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "schedule_knobs or full_1080 or image_out" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
step tests $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "schedule_knobs or full_1080" -x -q --timeout 200 --timeout-method thread \
    --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/tests_checked.log 2>&1
step tests_checked $?
ROUNDS=5 bash tools/calls/gpu_r05_ab.sh $O/ab rec=bevy_raytrace_amd/librt_hip_rec.so cur=product l4r96=product:block_lead=4,block_region=96
step ab $?
for pass in 1 2; do
  for nk in "8 7" "4 3" "2 1"; do
    for t in "" block_lead=0; do
      PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 $nk 20 >> $O/shards.log 2>&1
      step "shard $nk $pass $t" $?
    done
  done
done
exit 0
