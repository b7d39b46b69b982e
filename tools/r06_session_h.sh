#!/bin/bash
# round-6 session h: GPU suite (single-pass voting scans), refine stage on B / 0600, then session g
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r06h || exit 1
for wl in "--pairs 16 --concurrency 8 --single 10" "--png 0600-Left.png 0600-Right.png --pairs 16 --concurrency 8 --single 5"; do
  timeout -k 10 200 python3 tools/stage_probe.py $wl --label r06h 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06h_stage.txt || exit 1
done
bash tools/r06_session_g.sh
