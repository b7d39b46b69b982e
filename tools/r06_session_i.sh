#!/bin/bash
# round-6 session i: aggregation stores plain vs non-temporal (agg_plain_st) on B, 0600, C, E
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
WL=("--pairs 32 --concurrency 16"
    "--png 0600-Left.png 0600-Right.png --pairs 16 --concurrency 8"
    "--height 1000 --width 1500 --max-disparity 256 --pairs 8 --concurrency 4"
    "--height 1536 --width 2048 --max-disparity 320 --grey --pairs 4 --concurrency 2")
for r in 1 2; do
  for wl in "${WL[@]}"; do
    for x in default agg_plain_st; do
      if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
      timeout -k 10 200 python3 tools/stage_probe.py $wl --label $x 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06i_stage.txt || exit 1
    done
  done
done
