#!/bin/bash
# GPU box, round-4 session 9: the C++ API programs (cv::Mat forms of the matcher and of
# f2-f4) and the full GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_cpp_api.py -v --timeout 120 --timeout-method thread > gpurun_out/r04i_cpp.log 2>&1
rc=$?; echo "cpp rc=$rc: $(tail -1 gpurun_out/r04i_cpp.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r04i_cpp.log | head -20; exit $rc; }
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04i_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04i_tests.log)"; exit $rc
