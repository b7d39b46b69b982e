#!/bin/bash
# round-6 session ad: XCD placement of the aggregation streamer's blocks per handle
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TSM_EXPERIMENT_LIB=build/exp/agg_xcc/libtsm_adcensus.so timeout -k 10 400 python3 tools/xcc_probe.py --handles 6 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee gpurun_out/r06ad.txt
