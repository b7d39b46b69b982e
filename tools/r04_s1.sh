#!/bin/bash
# GPU box, round-4 first session: the L3 probe, smoke + GPU suite + bench (r04_check.sh),
# then the XCD-remap A/B, the per-kernel PMC bytes and the single-frame timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/l3_probe > gpurun_out/r04a_l3_probe.txt 2>&1; rc=$?; echo "l3 rc=$rc"; cat gpurun_out/r04a_l3_probe.txt; [ $rc -ne 0 ] && exit $rc
bash tools/r04_check.sh r04a || exit $?
bash tools/lib_ab.sh noremap 2 || exit $?
bash tools/pmc_all.sh r04a || exit $?
bash tools/lat_trace.sh r04a || exit $?
