#!/bin/bash
# GPU box: same-box A/B of an environment switch over tools/stage_probe.py workloads.
#   tools/ab_env.sh "VAR=value" [reps]   -> rows "default" and "VAR=value" per workload, alternating
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
SW=$1; REPS=${2:-2}
WL=("--png 0600-Left.png 0600-Right.png --pairs 32 --concurrency 16 --single 5"
    "--pairs 128 --concurrency 64 --single 5"
    "--noisy --pairs 128 --concurrency 64 --single 5"
    "--hsi --pairs 64 --concurrency 32 --single 5"
    "--png Motorcycle_Left.png Motorcycle_Right.png --max-disparity 256 --pairs 16 --concurrency 8 --single 3")
for r in $(seq $REPS); do
  for wl in "${WL[@]}"; do
    timeout -k 10 200 python3 tools/stage_probe.py $wl --label default 2>&1 | grep -v "^\[" | tail -1 || exit 1
    timeout -k 10 200 env $SW python3 tools/stage_probe.py $wl --label "$SW" 2>&1 | grep -v "^\[" | tail -1 || exit 1
  done
done
