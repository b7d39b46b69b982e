#!/bin/bash
# GPU box, round-4 session 14: the cost walk without the in-loop store drain (the tail
# store's lane id recomputed instead of spilled): the full GPU suite, then a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/s14_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/s14_tests.log; exit 1; }
tail -2 gpurun_out/s14_tests.log
bash tools/exp_stage.sh
