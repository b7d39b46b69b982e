#!/bin/bash
# round-6 session n: GPU suite (fused discontinuity / refinement tail), refine stage, frame timeline
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r06x || exit 1
for wl in "--pairs 16 --concurrency 8 --single 10" "--png 0600-Left.png 0600-Right.png --pairs 16 --concurrency 8 --single 5" "--noisy --pairs 16 --concurrency 8 --single 10"; do
  timeout -k 10 200 python3 tools/stage_probe.py $wl --label r06x 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06x_stage.txt || exit 1
done
bash tools/lat_trace.sh r06x
