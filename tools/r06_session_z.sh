#!/bin/bash
# round-6 session z: per-pass scanline times with one pipeline alone (kernel trace of
# stage_probe, groups of one) on B_noisy and the 0600 pair, beside tools/micro/walk_probe
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for cfg in noisy real; do
  if [ $cfg = noisy ]; then ARGS="--noisy --pairs 4 --concurrency 1"; else ARGS="--png 0600-Left.png 0600-Right.png --pairs 4 --concurrency 1"; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z_$cfg -o run -- python3 tools/stage_probe.py $ARGS > gpurun_out/z_$cfg.log 2>&1 || { echo "rc=$? $cfg"; tail -5 gpurun_out/z_$cfg.log; exit 1; }
  tail -1 gpurun_out/z_$cfg.log
  S=$(ls gpurun_out/z_$cfg/run_kernel_stats.csv gpurun_out/z_$cfg/*/run_kernel_stats.csv 2>/dev/null | head -1)
  grep scan_line $S | cut -c1-200
done
