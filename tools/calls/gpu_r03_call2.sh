# round-3 GPU call 2: op_sel/MFMA isolation ubench, MFMA counter semantics,
# culled wall-time A/B (round-2 build vs this build), driver-form PMC passes
# (one 20-frame launch) and the rocprof kernel stats of the driver-form bench.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 180 ./tools/ubench/opsel_mfma 3 > gpurun_out/opsel_mfma.log 2>&1 || exit 21
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F16 GRBM_GUI_ACTIVE -d $R/gpurun_out/mfma_count -o run --output-format csv -- $R/tools/ubench/mfma_count > $R/gpurun_out/mfma_count.log 2>&1 || exit 22
cd $R
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --lib tools/librt_cur_tag.so > gpurun_out/ab_r02.json 2> gpurun_out/ab_r02.err || exit 23
timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 > gpurun_out/ab_r03.json 2> gpurun_out/ab_r03.err || exit 24
FPL=20 timeout -k 10 900 bash tools/pmc_round.sh > gpurun_out/pmc_round.log 2>&1 || exit 25
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/stats -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 20 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 > $R/gpurun_out/stats_bench.json 2> $R/gpurun_out/stats_bench.err || exit 26
