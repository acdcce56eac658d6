# round 5, call 17: the 8K frame on one GPU with the s_setprio rotation on /
# off (2 rounds each).  usage: bash tools/gpu_r05_call17.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
ROUNDS=2 bash tools/gpu_r05_ab.sh $O/ab8k p1=product:prio_mode=1 p0=product:prio_mode=0 \
    -- --config rtiow8k --frames-per-launch 1 --steps 1 --warmup 0
step ab8k $?
exit 0
