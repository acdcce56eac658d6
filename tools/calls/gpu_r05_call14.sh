# round 5, call 14: headline A/B of the walk issuing both halves' MFMAs back
# to back (-DRT_WALK_BOTH build) and of the tail / priority knobs at the
# call-sized block region.  usage: bash tools/calls/gpu_r05_call14.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash tools/calls/gpu_r05_ab.sh $O/ab base=tools/librt_r04_final.so cur=product both=tools/librt_r05_both.so \
    t05=product:tail=0/0.5/1 t2=product:tail=0/2/1 t105=product:tail=0/1/0.5 prio0=product:prio_mode=0
step ab $?
exit 0
