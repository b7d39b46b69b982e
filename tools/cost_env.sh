#!/bin/bash
# GPU box: the cost launch's average duration (bench roofline phase, HIP events, one pair a
# launch) under environment settings, same box.  usage: cost_env.sh "X=0" "TSM_COST_MFMA=1" ...
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ops --batch 16 --concurrency 16 > gpurun_out/cv_$i.log 2>&1 || { echo "[$kv] rc=$?"; tail -5 gpurun_out/cv_$i.log; exit 1; }
  echo "[$kv] $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/cv_$i.log) $(grep -o '"value": [0-9.]*' gpurun_out/cv_$i.log | head -1)"
done
