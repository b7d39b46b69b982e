#!/bin/bash
# GPU box: per experiment build, one-pipeline stage times and the default bench's pairs/s.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for lib in default "$@"; do
  if [ $lib = default ]; then unset TSM_LIB; else export TSM_LIB=build/exp/$lib/libtsm_adcensus.so; fi
  timeout -k 10 120 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 4 > gpurun_out/ls_${lib}a.log 2>&1 || { echo "$lib rc=$?"; exit 1; }
  timeout -k 10 120 python3 bench.py --no-cpu-baseline > gpurun_out/ls_${lib}b.log 2>&1 || { echo "$lib rc=$?"; exit 1; }
  echo "$lib one-pipeline $(grep -o '"stage_ms_per_pair": {[^}]*}' gpurun_out/ls_${lib}a.log | head -1) | group8 $(grep -o '"value": [0-9.]*' gpurun_out/ls_${lib}b.log | head -1)"
done
