#!/bin/bash
# GPU box: pairs/s of the default build for several bench argument sets (quoted).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ops $a > gpurun_out/bs_$i.log 2>&1 || { echo "[$a] rc=$?"; tail -5 gpurun_out/bs_$i.log; exit 1; }
  echo "[$a] $(grep -o '"value": [0-9.]*' gpurun_out/bs_$i.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bs_$i.log | head -1)"
done
