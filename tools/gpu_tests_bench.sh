#!/bin/bash
# GPU box: full GPU test suite (stop on failure), then the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tb_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/tb_tests.log)"
[ $rc -ne 0 ] && { tail -40 gpurun_out/tb_tests.log; exit $rc; }
for c in "$@"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --concurrency $c > gpurun_out/tb_bench_c$c.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -20 gpurun_out/tb_bench_c$c.log; exit $rc; }
  echo "conc $c: $(grep -o '"value": [0-9.]*' gpurun_out/tb_bench_c$c.log) $(grep -o '"stage_ms_per_pair": {[^}]*}' gpurun_out/tb_bench_c$c.log) $(grep -o '"frac": [0-9.]*' gpurun_out/tb_bench_c$c.log)"
done
