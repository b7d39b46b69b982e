#!/bin/bash
# round-6 session l: GPU suite (HSI records with split colour words, plain BIG aggregation stores),
# then HSI / C / E stage times
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r06l || exit 1
for wl in "--hsi --pairs 32 --concurrency 16" "--height 1000 --width 1500 --max-disparity 256 --pairs 8 --concurrency 4" \
          "--hsi --pairs 32 --concurrency 16" "--pairs 32 --concurrency 16 --single 10"; do
  timeout -k 10 200 python3 tools/stage_probe.py $wl --label r06l 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06l_stage.txt || exit 1
done
