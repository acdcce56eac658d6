# round-4 GPU call 3: the tile epilogue's ORs as dual-issued v_bitop3_b32
# (and the queue entry's group index as one SGPR): same-box A/B against the
# build before it (tools/librt_r04_base.so), driver form, interleaved; the
# GPU suite on the new build; its PMC passes (one 20-frame launch).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04/c3
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
B="--steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
timeout -k 10 120 python -u bench.py $B --lib tools/librt_r04_base.so > $O/ab_warm.json 2>/dev/null
step warm $?
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py $B --lib tools/librt_r04_base.so > $O/ab_base_$i.json 2>/dev/null
  step "base $i" $?
  timeout -k 10 120 python -u bench.py $B > $O/ab_new_$i.json 2>/dev/null
  step "new $i" $?
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
step tests $?
FPL=20 bash tools/pmc_round.sh > $O/pmc_round.log 2>&1
step pmc $?
mv gpurun_out/pmc_* $O/ 2>/dev/null
exit 0
