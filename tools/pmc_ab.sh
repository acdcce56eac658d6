#!/bin/bash
# VALU / SALU instruction counts of rt_render_kernel for two library builds
# (one rocprofv3 --pmc pass each, same frame): does a change cut the VALU stream?
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM \
      -d "$R/gpurun_out/pmcab_$i" -o run --output-format csv -- \
      python3 "$R/tools/ab.py" "$R/$lib" --reps 1 > "$R/gpurun_out/pmcab_$i.log" 2>&1
  rc=$?; echo "pass $i ($lib) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
