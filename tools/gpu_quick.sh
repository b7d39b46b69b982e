#!/bin/bash
# GPU box: parity tests (stop on failure), then a concurrency-1 kernel trace of the
# in-tree library and, optionally, of TSM_AGG_KERNEL variants ("dma", "stream", "split").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/q_tests.log)"
[ $rc -ne 0 ] && { tail -30 gpurun_out/q_tests.log; exit $rc; }
for k in cur "$@"; do
  if [ "$k" = cur ]; then unset TSM_AGG_KERNEL; else export TSM_AGG_KERNEL=$k; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/q_$k -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 2 > gpurun_out/q_$k.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "trace $k rc=$rc"; tail -5 gpurun_out/q_$k.log; exit $rc; }
  echo "== $k"; python3 tools/trace_agg.py gpurun_out/q_$k/run_kernel_trace.csv > gpurun_out/q_$k.txt; head -8 gpurun_out/q_$k.txt
  grep -o '"value": [0-9.]*' gpurun_out/q_$k.log
done
