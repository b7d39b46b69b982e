#!/bin/bash
# GPU box: parity tests with an environment setting, then bench (default group size and
# one pipeline) alternating default / setting.  usage: env_ab.sh VAR=value [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
KV=$1; shift
env $KV timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api_contract.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/eab_tests.log 2>&1
rc=$?; echo "tests($KV) rc=$rc: $(tail -1 gpurun_out/eab_tests.log)"
[ $rc -ne 0 ] && { tail -30 gpurun_out/eab_tests.log; exit $rc; }
for r in 1 2; do
  for mode in default set; do
    if [ $mode = default ]; then E=""; else E=$KV; fi
    env $E timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/eab_${mode}_$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $mode rc=$rc"; tail -20 gpurun_out/eab_${mode}_$r.log; exit $rc; }
    echo "$mode r$r: $(grep -o '"value": [0-9.]*' gpurun_out/eab_${mode}_$r.log | head -1) $(grep -o '"stage_ms_per_pair": {[^}]*}' gpurun_out/eab_${mode}_$r.log)"
  done
done
