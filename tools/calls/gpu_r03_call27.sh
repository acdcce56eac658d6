# round-3 GPU call 27: driver-form bench A/B, the slot-buffer kernel vs the
# build before it (tools/librt_base.so), interleaved, one box.
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
for i in 1 2 3; do
  timeout -k 10 200 $B --lib tools/librt_base.so > gpurun_out/abb_base_$i.json 2> gpurun_out/abb_base_$i.err || exit 271
  timeout -k 10 200 $B > gpurun_out/abb_new_$i.json 2> gpurun_out/abb_new_$i.err || exit 272
done
