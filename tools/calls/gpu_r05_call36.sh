# round 5: lead items after the pixel items (own grouped order). The
# the product and checked builds, a same-box A/B of lead sizes against the
# current plan (driver form, 3 rounds), and one WRITE_SIZE pass per arm.
# usage: bash tools/calls/gpu_r05_call36.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "schedule_knobs or block_order or full_1080" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
step tests $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k schedule_knobs -x -q --timeout 200 --timeout-method thread \
    --rt-lib bevy_raytrace_amd/librt_hip_checked.so > $O/tests_checked.log 2>&1
step tests_checked $?
bash tools/calls/gpu_r05_ab.sh $O/ab rec=bevy_raytrace_amd/librt_hip_rec.so cur=product l4=product:block_lead=4 l4r96=product:block_lead=4,block_region=96
step ab $?
cd /tmp && export TMPDIR=/tmp
for arm in "l4:--tune block_lead=4" "l4r96:--tune block_lead=4 --tune block_region=96"; do
  n=${arm%%:*}; t=${arm#*:}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$O/pmc_$n" -o run --output-format csv -- \
      python3 $R/bench.py --steps 20 --warmup 0 --frames-per-launch 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 $t > $O/pmc_$n.log 2>&1
  step "pmc $n" $?
done
exit 0
