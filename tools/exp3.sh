#!/bin/bash
# GPU box: one-pipeline stage times for experiment builds x aggregation kernels.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for k in split v7; do
for lib in default "$@"; do
  if [ $lib = default ]; then unset TSM_LIB; else export TSM_LIB=build/exp/$lib/libtsm_adcensus.so; fi
  TSM_AGG_KERNEL=$k timeout -k 10 120 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 4 > gpurun_out/e3_${k}_$lib.log 2>&1 || exit $?
  echo "$k $lib $(grep -o '"aggregate": [0-9.]*' gpurun_out/e3_${k}_$lib.log | head -1)"
done
done
