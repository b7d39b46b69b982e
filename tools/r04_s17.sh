#!/bin/bash
# GPU box, round-4 session 17: group size of the batch (pairs per group, two group streams)
# on one box: 64 (default) against 32 and 48, alternating, short bench runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for k in 64 32 48; do
    timeout -k 10 240 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-ops --no-configs --concurrency $k > gpurun_out/s17_$k.log 2>&1 || { echo "k=$k rc=$?"; tail -5 gpurun_out/s17_$k.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/s17_$k.log') if l.startswith('{')][-1]); print('conc $k', d['value'], d['ms_per_step'], d['verified'])"
  done
done
