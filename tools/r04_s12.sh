#!/bin/bash
# GPU box, round-4 session 12: the streamer's two-pixels-a-wave form (label slices of <= 32
# vectors): the full GPU suite, then per-pair stage times at config C's and E's sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/s12_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/s12_tests.log; exit 1; }
tail -3 gpurun_out/s12_tests.log
: > gpurun_out/s12.txt
run() {
  timeout -k 10 240 python3 tools/stage_probe.py --label pw2 "$@" >> gpurun_out/s12.txt 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/s12.txt; exit 1; }
  tail -1 gpurun_out/s12.txt
}
run --height 1000 --width 1500 --max-disparity 256 --pairs 16 --concurrency 8
run --height 1536 --width 2048 --max-disparity 320 --pairs 8 --concurrency 4
run --pairs 64 --concurrency 32
# the cost walk without its volume stores (timing probe), against the default build
bash tools/exp_stage.sh costnostore
