#!/bin/bash
# round-6 session f: GPU suite + default bench on the CU-masked group streams
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r06f || exit 1
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r06f_bench.log 2>&1; rc=$?; echo bench rc=$rc
grep '^{' gpurun_out/r06f_bench.log | tail -1 > gpurun_out/r06f_bench.json
tail -c 2200 gpurun_out/r06f_bench.json
