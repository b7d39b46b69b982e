#!/bin/bash
# GPU box: single-frame latency (tools/latency.py) of the default library and experiment
# builds, alternating.  usage: lat_ab.sh <exp name> ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for x in default "$@"; do
    if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
    timeout -k 10 200 python3 tools/latency.py 1 > gpurun_out/lat_$x.log 2>&1 || { echo "$x rc=$?"; tail -5 gpurun_out/lat_$x.log; exit 1; }
    echo "$x r$r: $(tr '\n' ' ' < gpurun_out/lat_$x.log)"
  done
done
