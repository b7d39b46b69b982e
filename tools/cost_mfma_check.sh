#!/bin/bash
# GPU box: parity (stage dumps + configs) with the matrix-core cost build, then one-pipeline
# kernel traces of the cost stage with it (default) and with the walk (TSM_COST_MFMA=0),
# then default-bench pairs/s for both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/cm_tests.log 2>&1
rc=$?; echo "parity rc=$rc: $(tail -1 gpurun_out/cm_tests.log)"
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/cm_tests.log | head -20; tail -30 gpurun_out/cm_tests.log; exit $rc; }
for m in 1 0; do
  TSM_COST_MFMA=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cm_$m -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 2 > gpurun_out/cm_$m.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "trace $m rc=$rc"; tail -5 gpurun_out/cm_$m.log; exit $rc; }
  echo "== TSM_COST_MFMA=$m"; python3 tools/trace_agg.py gpurun_out/cm_$m/run_kernel_trace.csv > gpurun_out/cm_$m.txt; grep -E "cost|census" gpurun_out/cm_$m.txt
done
for r in 1 2; do
  for m in 1 0; do
    TSM_COST_MFMA=$m timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/cmb_${m}_$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $m rc=$rc"; tail -20 gpurun_out/cmb_${m}_$r.log; exit $rc; }
    echo "mfma=$m r$r: $(grep -o '"value": [0-9.]*' gpurun_out/cmb_${m}_$r.log | head -1) $(grep -o '"roofline": {[^}]*}' gpurun_out/cmb_${m}_$r.log)"
  done
done
