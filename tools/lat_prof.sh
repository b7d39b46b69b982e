#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/latency.py 1 > gpurun_out/lat1.log 2>&1 || { echo "lat rc=$?"; tail gpurun_out/lat1.log; exit 1; }
cat gpurun_out/lat1.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/latprof -o run -- python3 tools/latency.py 1 > gpurun_out/latprof.log 2>&1
echo "prof rc=$?"
