#!/bin/bash
# round-6 session ac: handle-to-handle spread of the headline batch (8 fresh handles a process)
# with the pair slots padded by 0 / 68 KB / 2 MB + 12 KB (build/exp/slot_pad, TSM_SLOT_PAD)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TSM_EXPERIMENT_LIB=build/exp/slot_pad/libtsm_adcensus.so
for pad in 0 69632 2109440 0 69632 2109440; do
  echo "== pad $pad"
  TSM_SLOT_PAD=$pad timeout -k 10 300 python3 tools/headline_ab.py --reps 6 --batches 3 --variants fresh 2>&1 | grep -v "WARNING\|amdgpu.ids" || exit 1
done 2>&1 | tee gpurun_out/r06ac.txt
