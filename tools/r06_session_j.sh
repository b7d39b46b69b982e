#!/bin/bash
# round-6 session j: per-step stamps of the fused aggregation streamer (0600 pair, config B)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TSM_EXPERIMENT_LIB=build/exp/agg_stamps/libtsm_adcensus.so
timeout -k 10 200 python3 tools/agg_stamps.py 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee gpurun_out/r06j_stamps.txt || exit 1
timeout -k 10 200 python3 tools/agg_stamps.py --synthetic 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06j_stamps.txt || exit 1
timeout -k 10 200 python3 tools/agg_stamps.py --png Motorcycle_Left.png Motorcycle_Right.png --max-disparity 256 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06j_stamps.txt || exit 1
