# round 5, call 22: the pair-balanced final drain (-DRT_DRAIN_PAIR build,
# tools/librt_r05_pair.so): the GPU suite on it, then the headline and rtiow4k
# A/B against the product and the round-4 library.
# usage: bash tools/calls/gpu_r05_call22.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    --rt-lib tools/librt_r05_pair.so --deselect tests/test_gpu_parity.py::test_native_library_is_in_tree \
    > $O/gpu_tests_pair.log 2>&1
step tests $?
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product pair=tools/librt_r05_pair.so
step ab $?
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab4k cur=product pair=tools/librt_r05_pair.so \
    -- --config rtiow4k --frames-per-launch 1 --steps 1 --warmup 1
step ab4k $?
for t in "" ; do
  PROBE_LIB=tools/librt_r05_pair.so timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard8.log 2>&1
  step "shard8 pair" $?
  timeout -k 10 120 python -u tools/split_probe.py 20 8 7 20 >> $O/shard8.log 2>&1
  step "shard8 cur" $?
done
exit 0
