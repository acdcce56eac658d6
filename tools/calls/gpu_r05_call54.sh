# round 5: the N = 4 / 2 row shards (their last shard, split_probe) with the
# end-of-launch chunks of 32 against 16 (a build of the same sources), and
# the N = 8 shard's lead size (2 by the call, against 3 / 4) with the final
# tail. 2 passes.  usage: bash tools/calls/gpu_r05_call54.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for pass in 1 2; do
  for nk in "4 3" "2 1"; do
    for lib in "" bevy_raytrace_amd/librt_hip_ct16.so; do
      PROBE_LIB=$lib timeout -k 10 120 python -u tools/split_probe.py 20 $nk 20 > $O/shard_$(echo $nk | tr ' ' _)_$(basename ${lib:-product})_$pass.log 2>&1
      step "shard $nk $lib $pass" $?
    done
  done
  for t in "" block_lead=3 block_lead=4; do
    PROBE_TUNE=$t timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard8_lead.log 2>&1
    step "shard8 $t $pass" $?
  done
done
exit 0
