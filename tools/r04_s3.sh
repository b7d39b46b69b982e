#!/bin/bash
# GPU box, round-4 session 3: GPU suite on the restructured split streamer, then stage
# timings: new default, round-3 base, base + 40 SALU a step (probe), new + split streamer
# for the single passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04c_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/r04c_tests.log | head -20; tail -30 gpurun_out/r04c_tests.log; exit $rc; }
bash tools/exp_stage.sh r04base salu40 v6all
