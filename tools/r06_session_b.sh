#!/bin/bash
# round-6 session b: headline A/B (long-lived vs fresh handle vs OMP20), kernel stats of each
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/headline_ab.py --reps 3 --batches 5 2>&1 | grep -v WARNING | tee gpurun_out/r06b_ab.txt || exit 1
for v in fresh omp20; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06b_prof_$v -o run -- python3 tools/headline_ab.py --reps 1 --batches 3 --variants $v > gpurun_out/r06b_prof_$v.log 2>&1 || exit 1
done
for v in fresh omp20; do echo == $v; head -12 gpurun_out/r06b_prof_$v/run_kernel_stats.csv | cut -c1-160; done
