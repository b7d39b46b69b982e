#!/bin/bash
# round-6 session d: CU-masked group streams -- queue ids and the handle A/B
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/headline_ab.py --reps 2 --batches 4 --variants fresh,long,fresh 2>&1 | grep -v WARNING | tee gpurun_out/r06d_ab.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06d_prof -o run -- python3 tools/headline_ab.py --reps 2 --batches 2 --variants long,fresh > gpurun_out/r06d_prof.log 2>&1 || exit 1
grep round gpurun_out/r06d_prof.log
