#!/bin/bash
# GPU box: default bench pairs/s and one-pipeline stage times, alternating the default
# library and an experiment build (same box).  usage: lib_ab.sh <exp name> [rounds]
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
X=$1; R=${2:-2}
for r in $(seq 1 $R); do
  for lib in tea_stereo_matching_amd/lib/libtsm_adcensus.so build/exp/$X/libtsm_adcensus.so; do
    n=$(basename $(dirname $lib))
    TSM_EXPERIMENT_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ops --no-configs > gpurun_out/lab_${n}_$r.log 2>&1 || { echo "$n rc=$?"; tail -5 gpurun_out/lab_${n}_$r.log; exit 1; }
    echo "$n r$r: $(grep -o '"value": [0-9.]*' gpurun_out/lab_${n}_$r.log | head -1) $(grep -o '"aggregate": [0-9.]*' gpurun_out/lab_${n}_$r.log | head -1)"
  done
done
