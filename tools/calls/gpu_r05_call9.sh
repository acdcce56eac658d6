# round 5, call 9: item order A/B (pixel-major vs grouped by 8 / by 4) and
# the render kernel's WRITE_SIZE per 20-frame launch for each.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product grp8=product:item_order=7 \
    grp4=product:item_order=7,pix_group=4
step ab $?
cd /tmp && export TMPDIR=/tmp
for arm in "o3:item_order=3" "g8:item_order=7" "g4:item_order=7 --tune pix_group=4"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/$O/pmcw_${arm%%:*} -o run \
      --output-format csv -- python3 $R/bench.py --steps 20 --warmup 0 --frames-per-launch 20 \
      --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --tune ${arm#*:} > $R/$O/pmcw_${arm%%:*}.log 2>&1
  step "pmc write ${arm%%:*}" $?
done
exit 0
