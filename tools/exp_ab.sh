#!/bin/bash
# GPU box: parity tests against an experiment build, then bench pairs/s for the default
# and experiment builds (alternating, 2 rounds).  usage: exp_ab.sh <exp-name> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
X=$1; shift
TSM_EXPERIMENT_LIB=build/exp/$X/libtsm_adcensus.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab_${X}_tests.log 2>&1
rc=$?; echo "tests($X) rc=$rc: $(tail -1 gpurun_out/ab_${X}_tests.log)"
[ $rc -ne 0 ] && { tail -30 gpurun_out/ab_${X}_tests.log; exit $rc; }
for r in 1 2; do
  for lib in default $X; do
    if [ $lib = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$lib/libtsm_adcensus.so; fi
    timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/ab_${lib}_$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $lib rc=$rc"; tail -20 gpurun_out/ab_${lib}_$r.log; exit $rc; }
    echo "$lib r$r: $(grep -o '"value": [0-9.]*' gpurun_out/ab_${lib}_$r.log | head -1) $(grep -o '"stage_ms_per_pair": {[^}]*}' gpurun_out/ab_${lib}_$r.log)"
  done
done
