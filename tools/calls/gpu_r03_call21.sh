# round-3 GPU call 21: candidate flags by v_perm_b32 and a branch-free queue
# append -- parity (intersect + render tests, smoke), A/B kernel time against
# the previous commit's build, VALU per segment (PMC).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_intersect.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_perm.log 2>&1 || exit 211
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_perm.log 2>&1 || exit 212
for i in 1 2; do
  PROBE_LIB=tools/librt_base.so timeout -k 10 200 python -u tools/item_probe.py 20 "" > gpurun_out/ab_perm_base_$i.log 2>&1 || exit 213
  timeout -k 10 200 python -u tools/item_probe.py 20 "" > gpurun_out/ab_perm_new_$i.log 2>&1 || exit 214
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_MFMA_F16 -d "$R/gpurun_out/spmc_perm" -o run --output-format csv -- python3 "$R/tools/shard_pmc.py" 8 > "$R/gpurun_out/spmc_perm.log" 2>&1 || exit 215
