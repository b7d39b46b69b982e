#!/bin/bash
# GPU box, round-4 first session: smoke + GPU suite + bench (r04_check.sh), then the
# XCD-remap A/B, the per-kernel PMC bytes and the single-frame timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r04_check.sh r04a || exit $?
bash tools/lib_ab.sh noremap 2 || exit $?
bash tools/pmc_all.sh r04a || exit $?
bash tools/lat_trace.sh r04a || exit $?
