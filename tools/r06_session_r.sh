#!/bin/bash
# round-6 session r: single-pass stamps (0600, Motorcycle), 8 window reads a round trip (A/B)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TSM_EXPERIMENT_LIB=build/exp/agg_stamps_single/libtsm_adcensus.so
timeout -k 10 200 python3 tools/agg_stamps.py 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee gpurun_out/r06r_stamps_single.txt || exit 1
timeout -k 10 200 python3 tools/agg_stamps.py --png Motorcycle_Left.png Motorcycle_Right.png --max-disparity 256 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06r_stamps_single.txt || exit 1
unset TSM_EXPERIMENT_LIB
WL=("--png 0600-Left.png 0600-Right.png --pairs 16 --concurrency 8" "--pairs 32 --concurrency 16"
    "--png Motorcycle_Left.png Motorcycle_Right.png --max-disparity 256 --pairs 8 --concurrency 4" "--hsi --pairs 32 --concurrency 16")
for r in 1 2; do
  for wl in "${WL[@]}"; do
    for x in default agg_read8; do
      if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
      timeout -k 10 200 python3 tools/stage_probe.py $wl --label $x 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06r_stage.txt || exit 1
    done
  done
done
