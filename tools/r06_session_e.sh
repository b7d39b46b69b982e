#!/bin/bash
# round-6 session e: arena placement -- default allocation vs physically contiguous arenas
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for x in default alloc_contig default alloc_contig; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  echo "== $x"
  timeout -k 10 300 python3 tools/headline_ab.py --reps 2 --batches 4 --variants fresh,long,fresh 2>&1 | grep -v "WARNING\|amdgpu.ids" || exit 1
done 2>&1 | tee gpurun_out/r06e_ab.txt
