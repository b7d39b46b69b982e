#!/bin/bash
# round-6 session ah: horizontal pass with LDS-staged side rows and every vector stored
# without a branch (build/exp/scan_hrows_uncond) against the product, one pipeline alone;
# then a kernel trace of each on the 0600 pair (per-pass times)
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in tea_stereo_matching_amd/lib/libtsm_adcensus.so build/exp/scan_hrows_uncond/libtsm_adcensus.so; do
    n=$(basename $(dirname $lib))
    for wl in "--noisy --pairs 8 --concurrency 8" "--png 0600-Left.png 0600-Right.png --pairs 8 --concurrency 8"; do
      TSM_EXPERIMENT_LIB=$lib timeout -k 10 200 python3 tools/stage_probe.py $wl --label "$n" 2>&1 | grep -v "WARNING\|amdgpu.ids" || exit 1
    done
  done
done
for lib in tea_stereo_matching_amd/lib/libtsm_adcensus.so build/exp/scan_hrows_uncond/libtsm_adcensus.so; do
  n=$(basename $(dirname $lib))
  TSM_EXPERIMENT_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ah_$n -o run -- python3 tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 4 --concurrency 1 > gpurun_out/ah_$n.log 2>&1 || { echo "rc=$?"; exit 1; }
  S=$(ls gpurun_out/ah_$n/run_kernel_stats.csv gpurun_out/ah_$n/*/run_kernel_stats.csv 2>/dev/null | head -1)
  echo "== $n"; grep scan_line $S | cut -d, -f1,2,4 | cut -c1-140
done
