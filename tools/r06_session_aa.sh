#!/bin/bash
# round-6 session aa: horizontal scanline passes with their colour-difference rows staged in
# LDS -- GPU suite, then per-pair stage times (one pipeline) and the headline, alternating
# the product library and the previous form (build/exp/scan_hrows_off)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r06aa || exit 1
for r in 1 2; do
  for lib in tea_stereo_matching_amd/lib/libtsm_adcensus.so build/exp/scan_hrows_off/libtsm_adcensus.so; do
    n=$(basename $(dirname $lib))
    for wl in "--noisy --pairs 8 --concurrency 8" "--png 0600-Left.png 0600-Right.png --pairs 8 --concurrency 8" "--pairs 16 --concurrency 8"; do
      TSM_EXPERIMENT_LIB=$lib timeout -k 10 200 python3 tools/stage_probe.py $wl --label "$n" 2>&1 | grep -v "WARNING\|amdgpu.ids" || exit 1
    done
  done
done
bash tools/lib_ab.sh scan_hrows_off 2
