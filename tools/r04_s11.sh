#!/bin/bash
# GPU box, round-4 session 11: the HSI cost walk's parity tests, then aggregation probes at
# config C's and E's sizes and in HSI (tools/stage_probe.py: pairs/s, per-pair stage times
# with one pipeline alone); the experiment builds are timing probes (outputs unchecked).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "hsi or HSI or mask or full_size" > gpurun_out/s11_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/s11_tests.log; exit 1; }
tail -2 gpurun_out/s11_tests.log
run() {  # experiment name, stage_probe args...
  local x=$1; shift
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  timeout -k 10 240 python3 tools/stage_probe.py --label $x "$@" >> gpurun_out/s11.txt 2>&1 || { echo "$x rc=$?"; tail -5 gpurun_out/s11.txt; exit 1; }
  tail -1 gpurun_out/s11.txt
}
: > gpurun_out/s11.txt
run default --hsi --pairs 64 --concurrency 32
# per-step work: one label slice of 49 (D=192) or 33 (D=128) lanes against two of 33 / 32 (D=256)
for d in 256 192 128; do run default --height 1000 --width 1500 --max-disparity $d --pairs 16 --concurrency 8; done
for x in nostore win1; do run $x --height 1000 --width 1500 --max-disparity 256 --pairs 16 --concurrency 8; done
for x in nostore win1; do run $x --hsi --pairs 64 --concurrency 32; done
for x in default nostore; do run $x --height 1536 --width 2048 --max-disparity 320 --pairs 8 --concurrency 4; done
