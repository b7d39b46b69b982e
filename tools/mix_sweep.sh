#!/bin/bash
# GPU box: for each quoted env setting, the GPU parity suite under that setting, then the
# default bench (group launches) and a one-pipeline bench.  usage: mix_sweep.sh "A=1 B=2" ...
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/mx_${i}_t.log 2>&1 || { echo "[$kv] tests rc=$?"; tail -15 gpurun_out/mx_${i}_t.log; exit 1; }
  env $kv timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ops > gpurun_out/mx_${i}_b.log 2>&1 || { echo "[$kv] bench rc=$?"; tail -5 gpurun_out/mx_${i}_b.log; exit 1; }
  env $kv timeout -k 10 120 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-ops --concurrency 1 --batch 4 > gpurun_out/mx_${i}_a.log 2>&1 || { echo "[$kv] bench1 rc=$?"; tail -5 gpurun_out/mx_${i}_a.log; exit 1; }
  echo "[$kv] $(tail -1 gpurun_out/mx_${i}_t.log) | group $(grep -o '"value": [0-9.]*' gpurun_out/mx_${i}_b.log | head -1) $(grep -o '"aggregate": [0-9.]*' gpurun_out/mx_${i}_b.log | tail -1) | one-pipeline $(grep -o '"aggregate": [0-9.]*' gpurun_out/mx_${i}_a.log | head -1)"
done
