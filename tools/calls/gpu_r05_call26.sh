# round 5, call 26: tail 0,1,0.5 against the default 0,1,1 on whole frames:
# the headline, spheres10k1080 and rtiow4k.  usage: bash tools/calls/gpu_r05_call26.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab cur=product t105=product:tail=0/1/0.5
step ab $?
ROUNDS=3 bash tools/calls/gpu_r05_ab.sh $O/ab10k cur=product t105=product:tail=0/1/0.5 \
    -- --config spheres10k1080 --frames-per-launch 2 --steps 2 --warmup 1
step ab10k $?
ROUNDS=2 bash tools/calls/gpu_r05_ab.sh $O/ab4k cur=product t105=product:tail=0/1/0.5 \
    -- --config rtiow4k --frames-per-launch 1 --steps 1 --warmup 1
step ab4k $?
exit 0
