#!/bin/bash
# GPU box: pairs/s for (group streams, batch, group size) settings, same box.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
run() { env $1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ops $2 > gpurun_out/gs.log 2>&1 || { echo "[$1 $2] rc=$?"; tail -3 gpurun_out/gs.log; exit 1; }; echo "[$1 $2] $(grep -o '"value": [0-9.]*' gpurun_out/gs.log | head -1)"; }
for a in "$@"; do run "${a%%|*}" "${a#*|}"; done
