# Forward bound rows: GPU suite on the in-tree build, then the timing A/B
# against the previous build and the phase profile.
# usage: bash tools/calls/gpu_r04_fwd.sh <out dir> <baseline lib>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/calls/gpu_r04_sens.sh $O "$2" || exit $?
timeout -k 10 200 python -u tools/prof_phases.py 4,1,0 > $O/phases.log 2>&1
rc=$?; echo "== phases rc=$rc"; exit $rc
