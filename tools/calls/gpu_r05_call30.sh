# round 5, call 30: block region 64 (the call's rule at the headline) against
# 56 / 52 / 48 with the final tail: time (driver form) and the render
# kernel's WRITE_SIZE per 20-frame launch.  usage: bash tools/calls/gpu_r05_call30.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab cur=product b56=product:block_region=56 b52=product:block_region=52 \
    b48=product:block_region=48
step ab $?
cd /tmp && export TMPDIR=/tmp
for arm in "b64:block_region=64" "b56:block_region=56" "b52:block_region=52" "b48:block_region=48"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/$O/pmcw_${arm%%:*} -o run \
      --output-format csv -- python3 $R/bench.py --steps 20 --warmup 0 --frames-per-launch 20 \
      --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --tune ${arm#*:} > $R/$O/pmcw_${arm%%:*}.log 2>&1
  step "pmc write ${arm%%:*}" $?
done
exit 0
