#!/bin/bash
# round-6 session ag: handle spread with one group of 128 pairs (one arena, one stream)
# against two groups of 64 (two arenas on two streams), 6 fresh handles a process each
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for c in 64 128 64 128 43; do
  echo "== concurrency $c"
  timeout -k 10 400 python3 tools/xcc_probe.py --handles 6 --concurrency $c 2>&1 | grep -v "WARNING\|amdgpu.ids" | sed 's/; *$//' || exit 1
done | tee gpurun_out/r06ag.txt
