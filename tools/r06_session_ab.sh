#!/bin/bash
# round-6 session ab: kernel trace of the headline handle A/B (fresh / long / fresh handles):
# which handles' group streams overlap
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_prof -o run -- python3 tools/headline_ab.py --reps 2 --batches 4 --variants fresh,long,fresh > gpurun_out/ab_prof.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/ab_prof.log; exit 1; }
grep round gpurun_out/ab_prof.log
K=$(ls gpurun_out/ab_prof/run_kernel_trace.csv gpurun_out/ab_prof/*/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/stream_overlap.py $K 100
