# round 5, call 10: block region (single-block items before the tail) at
# 96 / 64 / 48 samples x depth per lane with the grouped-by-4 item order:
# time and the render kernel's WRITE_SIZE per 20-frame launch.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product br64=product:block_region=64 \
    br48=product:block_region=48
step ab $?
cd /tmp && export TMPDIR=/tmp
for arm in "b96:block_region=96" "b64:block_region=64" "b48:block_region=48"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/$O/pmcw_${arm%%:*} -o run \
      --output-format csv -- python3 $R/bench.py --steps 20 --warmup 0 --frames-per-launch 20 \
      --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --tune ${arm#*:} > $R/$O/pmcw_${arm%%:*}.log 2>&1
  step "pmc write ${arm%%:*}" $?
done
exit 0
