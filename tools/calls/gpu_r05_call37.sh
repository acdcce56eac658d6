# round 5: lead sizes and block regions with the lead items after the pixel
# items (call 36 follow-up): a same-box A/B of 5 rounds against the recorded
# kernel, one WRITE_SIZE pass per lead arm.  usage: bash tools/calls/gpu_r05_call37.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=5 bash tools/calls/gpu_r05_ab.sh $O/ab rec=bevy_raytrace_amd/librt_hip_rec.so l4=product:block_lead=4 \
    l5=product:block_lead=5 l3=product:block_lead=3 l4r80=product:block_lead=4,block_region=80 l6r96=product:block_lead=6,block_region=96
step ab $?
cd /tmp && export TMPDIR=/tmp
for arm in "l5:--tune block_lead=5" "l3:--tune block_lead=3" "l4r80:--tune block_lead=4 --tune block_region=80" "l6r96:--tune block_lead=6 --tune block_region=96"; do
  n=${arm%%:*}; t=${arm#*:}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$O/pmc_$n" -o run --output-format csv -- \
      python3 $R/bench.py --steps 20 --warmup 0 --frames-per-launch 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 $t > $O/pmc_$n.log 2>&1
  step "pmc $n" $?
done
exit 0
