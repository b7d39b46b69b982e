#!/bin/bash
# GPU box: aggregation stage time per pair (one pipeline) for experiment builds.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TSM_AGG_KERNEL=${TSM_AGG_KERNEL:-split}
for lib in default "$@"; do
  if [ $lib = default ]; then unset TSM_LIB; else export TSM_LIB=build/exp/$lib/libtsm_adcensus.so; fi
  timeout -k 10 120 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 4 > gpurun_out/e2_$lib.log 2>&1 || exit $?
  echo "$lib $(grep -o '"stage_ms_per_pair": {[^}]*}' gpurun_out/e2_$lib.log)"
done
