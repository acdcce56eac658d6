# round 5, call 4: GPU suite on the product build (chunk-level bounds,
# grouped item order code), headline A/B (round-4 kernel, product with item
# order 3 / 7, LDS records with queue cap 9, cap 9 alone), 10k-sphere A/B
# (chunk bounds on / off), and WRITE_SIZE of one 20-frame launch per order.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab --tests base=tools/librt_r04_final.so cur=product \
    grp=product:item_order=7 lds9=tools/librt_r05_lds9.so cap9=tools/librt_r05_cap9.so
step ab $?
bash tools/calls/gpu_r05_ab.sh $O/ab10k base=tools/librt_r04_final.so cur=product notop=product:mf_top=0 \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
cd /tmp && export TMPDIR=/tmp
for arm in "o3:item_order=3" "o7:item_order=7"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/$O/pmcw_${arm%%:*} -o run \
      --output-format csv -- python3 $R/bench.py --steps 20 --warmup 0 --frames-per-launch 20 \
      --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --tune ${arm#*:} > $R/$O/pmcw_${arm%%:*}.log 2>&1
  step "pmc write ${arm%%:*}" $?
done
exit 0
