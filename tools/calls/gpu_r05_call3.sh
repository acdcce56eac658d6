# round 5, call 3: the GPU suite on the product build (bound-chunk loads
# without scratch spills), the A/B of the round-4 kernel against it and two
# variants (LDS records, queue cap 8), and the executed-work counters of the
# profile build with the diagnostic reductions timed apart.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab --tests base=tools/librt_r04_final.so cur=product \
    lds=tools/librt_r05_lds.so cap8=tools/librt_r05_cap8.so
step ab $?
timeout -k 10 300 python -u tools/executed.py $O/executed_raw.json > $O/executed.log 2>&1
step executed $?
exit 0
