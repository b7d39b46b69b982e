#!/bin/bash
# round-6 session q: GPU suite (label vectors dealt to ds_read_b128 lane groups), E / C / B / 0600 stages
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r06q || exit 1
for wl in "--height 1536 --width 2048 --max-disparity 320 --grey --pairs 4 --concurrency 2" \
          "--height 1000 --width 1500 --max-disparity 256 --pairs 8 --concurrency 4" \
          "--pairs 32 --concurrency 16" "--png 0600-Left.png 0600-Right.png --pairs 16 --concurrency 8"; do
  timeout -k 10 200 python3 tools/stage_probe.py $wl --label r06q 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06q_stage.txt || exit 1
done
