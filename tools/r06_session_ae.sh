#!/bin/bash
# round-6 session ae: is a handle's speed its memory or its queues?  6 fresh handles a
# process: as is / 30 GB of HBM held first (other physical pages) / 3 streams created first
# (other hardware queues)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TSM_EXPERIMENT_LIB=build/exp/agg_xcc/libtsm_adcensus.so
for v in "" "--shift-gb 30" "--streams 3" "--shift-gb 7" "--streams 1"; do
  echo "== $v"
  timeout -k 10 400 python3 tools/xcc_probe.py --handles 6 $v 2>&1 | grep -v "WARNING\|amdgpu.ids" | sed 's/; slot.*//' || exit 1
done | tee gpurun_out/r06ae.txt
