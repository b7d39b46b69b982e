#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for q in 4 8 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/hwq_$q.log 2>&1 || { echo "q=$q failed"; tail -5 gpurun_out/hwq_$q.log; exit 1; }
  echo "q=$q $(grep -o '"value": [0-9.]*' gpurun_out/hwq_$q.log | head -1)"
done
