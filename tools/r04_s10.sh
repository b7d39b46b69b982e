#!/bin/bash
# GPU box: partial-granule probe (784-B vectors vs granule multiples).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/granule_probe > gpurun_out/r04_granule_probe.txt 2>&1; rc=$?; cat gpurun_out/r04_granule_probe.txt; exit $rc
