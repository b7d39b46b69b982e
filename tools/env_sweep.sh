#!/bin/bash
# GPU box: for each quoted env setting (e.g. "TSM_AGG_KERNEL=v7 TSM_AGG_SLICES=2"), the
# one-pipeline stage times and the default bench's pairs/s.  usage: env_sweep.sh "A=1 B=2" ...
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 120 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 4 > gpurun_out/es_${i}a.log 2>&1 || { echo "[$kv] rc=$?"; tail -5 gpurun_out/es_${i}a.log; exit 1; }
  env $kv timeout -k 10 120 python3 bench.py --no-cpu-baseline > gpurun_out/es_${i}b.log 2>&1 || { echo "[$kv] rc=$?"; tail -5 gpurun_out/es_${i}b.log; exit 1; }
  echo "[$kv] one-pipeline $(grep -o '"aggregate": [0-9.]*' gpurun_out/es_${i}a.log | head -1) $(grep -o '"scanline": [0-9.]*' gpurun_out/es_${i}a.log | head -1) | group8 $(grep -o '"value": [0-9.]*' gpurun_out/es_${i}b.log | head -1)"
done
