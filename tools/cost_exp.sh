#!/bin/bash
# GPU box: the cost launch's average duration (bench roofline phase, HIP events, one pair
# per launch) for experiment builds of the library.  usage: cost_exp.sh base cm_STOREONLY ...
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for x in "$@"; do
  lib=build/exp/$x/libtsm_adcensus.so; [ "$x" = base ] && lib=tea_stereo_matching_amd/lib/libtsm_adcensus.so
  TSM_LIB=$lib timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ops --batch 16 --concurrency 16 > gpurun_out/ce_$x.log 2>&1 || { echo "$x rc=$?"; tail -5 gpurun_out/ce_$x.log; exit 1; }
  echo "$x $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/ce_$x.log)"
done
