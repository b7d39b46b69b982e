#!/bin/bash
# GPU box: smoke, then the GPU test suite (-v, every failure listed; per-test time limit).
# A fault / abort / timeout in smoke stops the script before the suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-suite}
shift || true
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/${TAG}_smoke.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python3 -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread "$@" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | grep -v PASSED | head -40
tail -3 gpurun_out/${TAG}_tests.log
exit $rc
