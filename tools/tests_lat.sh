#!/bin/bash
# GPU box: full GPU test suite (stop on failure), then single-frame latency (tools/latency.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-tl}
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/${TAG}_tests.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/${TAG}_tests.log | head -20; tail -30 gpurun_out/${TAG}_tests.log; exit $rc; }
timeout -k 10 200 python3 tools/latency.py 1 > gpurun_out/${TAG}_lat.log 2>&1
rc=$?; cat gpurun_out/${TAG}_lat.log; exit $rc
