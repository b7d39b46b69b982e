#!/bin/bash
# GPU box: GPU suite + single-frame latency, then the default bench's value and host legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/tests_lat.sh ${1:-pool} || exit $?
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-ops > gpurun_out/b_${1:-pool}.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b_${1:-pool}.log; exit 1; }
python3 - gpurun_out/b_${1:-pool}.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["value"], d["verified"], d["host_buffers"])
PY
