# round 5, call 1: where the headline kernel's wave time goes (rocprofv3
# stochastic PC sampling of one 8-frame launch; host-trap sampling if the
# stochastic method is refused), then the PMC passes of configs 3-5
# (tools/pmc_round.sh: 4K one frame, 10k spheres two frames, the 8K frame on
# one GPU).  usage: bash tools/calls/gpu_r05_call1.sh <out dir>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
export TMPDIR=/tmp
BCMD="python3 $R/bench.py --steps 8 --warmup 0 --frames-per-launch 8 --no-cpu-baseline --reuse-steps 0 --cull-steps 0"
timeout -k 10 180 rocprofv3 --kernel-trace --pc-sampling-beta-enabled --pc-sampling-method stochastic \
    --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv \
    -d $O/pcs_stoch -o ps -- $BCMD > $O/pcs_stoch.log 2>&1
rc=$?
echo "== pcs stochastic rc=$rc"
if fatal $rc; then exit $rc; fi
if [ $rc -ne 0 ]; then
  timeout -k 10 180 rocprofv3 --kernel-trace --pc-sampling-beta-enabled --pc-sampling-method host_trap \
      --pc-sampling-unit time --pc-sampling-interval 100 --output-format csv \
      -d $O/pcs_trap -o ps -- $BCMD > $O/pcs_trap.log 2>&1
  rc=$?
  echo "== pcs host_trap rc=$rc"
  if fatal $rc; then exit $rc; fi
fi
CFG=spheres10k1080 FPL=2 OUT=$O/pmc_10k bash tools/pmc_round.sh > $O/pmc_10k.log 2>&1
step pmc_10k $?
CFG=rtiow4k FPL=1 OUT=$O/pmc_4k bash tools/pmc_round.sh > $O/pmc_4k.log 2>&1
step pmc_4k $?
CFG=rtiow8k FPL=1 OUT=$O/pmc_8k bash tools/pmc_round.sh > $O/pmc_8k.log 2>&1
step pmc_8k $?
exit 0
