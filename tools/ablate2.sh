#!/bin/bash
# GPU box: default bench (batch 64, groups of 32) with stages skipped (experiment build,
# garbage results, timing only).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TSM_LIB=build/exp/skip/libtsm_adcensus.so
for s in 0 1 2 4 8 16; do
  TSM_SKIP=$s timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-ops > gpurun_out/ab2_$s.log 2>&1 || { echo "skip $s rc=$?"; exit 1; }
  echo "skip$s $(grep -o '"value": [0-9.]*' gpurun_out/ab2_$s.log)"
done
