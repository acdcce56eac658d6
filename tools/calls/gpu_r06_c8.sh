# round 6 call 8: the work chunk per atomic at the headline (knob wave_chunk,
# 5 rounds), and the 10,000-sphere workload at 2 / 6 / 12 frames per launch.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=5 CONFIGS="rtiow1080" bash tools/calls/gpu_r06_ab.sh $O base=product c96=product:wave_chunk=96 c128=product:wave_chunk=128 c160=product:wave_chunk=160
step ab $?
for f in 2 6 12; do
  timeout -k 10 300 python -u bench.py --config spheres10k1080 --steps $f --warmup 2 --frames-per-launch $f \
      --no-cpu-baseline --reuse-steps 0 --cull-steps 0 > $O/tenk_fpl$f.json 2>> $O/tenk.err
  step tenk_$f $?
done
exit 0
