# round-3 GPU call 15: N=8 rehearsal of the IPC path on one GPU (8 ranks,
# gloo for the control messages, every rank writing its rows into rank 0's
# mapped image): frames checksummed against N=1, config 1 and the 1080p frame.
set -o pipefail
mkdir -p gpurun_out
A="--steps 2 --warmup 1 --frames-per-launch 2 --no-cpu-baseline --reuse-steps 0 --cull-steps 0 --check"
timeout -k 10 200 python -u bench.py --config config1 $A > gpurun_out/n1_c1.json 2> gpurun_out/n8.err || exit 151
timeout -k 10 300 python -u bench.py --config config1 $A --gpus 8 --same-device --dist-backend gloo --gather ipc > gpurun_out/n8_c1.json 2>> gpurun_out/n8.err || exit 152
timeout -k 10 200 python -u bench.py $A > gpurun_out/n1_1080.json 2>> gpurun_out/n8.err || exit 153
timeout -k 10 300 python -u bench.py $A --gpus 8 --same-device --dist-backend gloo --gather ipc > gpurun_out/n8_1080.json 2>> gpurun_out/n8.err || exit 154
