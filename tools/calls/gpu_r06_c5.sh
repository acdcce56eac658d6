# round 6 call 5: tail / block-region knobs on the one-frame launches (time
# A/B + render-kernel WRITE_SIZE), and the scene-edit probe.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$(realpath -m $1)
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u tools/scene_edit_probe.py $O/scene_edit.json > $O/scene_edit.log 2>&1
step scene_edit $?
CONFIGS="rtiow4k spheres10k1080 rtiow1080" bash tools/calls/gpu_r06_ab.sh $O/ab base=product ts0=product:tail_split=0 br64=product:block_region=64 both=product:tail_split=0,block_region=64
step ab $?
ROUNDS=2 CONFIGS="rtiow8k" bash tools/calls/gpu_r06_ab.sh $O/ab base=product ts0=product:tail_split=0
step ab8k $?
cd /tmp && export TMPDIR=/tmp
for cfg in rtiow4k rtiow8k; do
  for arm in base ts0 both; do
    case $arm in base) T="" ;; ts0) T="--tune tail_split=0" ;; both) T="--tune tail_split=0 --tune block_region=64" ;; esac
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$O/pmc_${cfg}_$arm" -o run --output-format csv -- \
      python3 "$R/bench.py" --config $cfg --steps 1 --warmup 0 --frames-per-launch 1 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 $T > "$O/pmc_${cfg}_$arm.log" 2>&1
    step "pmc $cfg $arm" $?
  done
done
exit 0
