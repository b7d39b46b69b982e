#!/bin/bash
# round-6 session aj: f4 remap with LDS-staged windows (build/exp/remap_lds,
# tools/probes/remap_lds_stage.patch) -- stereo-ops GPU tests on that build, then the group
# remap against the product, alternating
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TSM_EXPERIMENT_LIB=build/exp/remap_lds/libtsm_adcensus.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stereo_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/aj_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/aj_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/aj_tests.log | head -20; exit $rc; }
for r in 1 2 3; do
  for lib in tea_stereo_matching_amd/lib/libtsm_adcensus.so build/exp/remap_lds/libtsm_adcensus.so; do
    n=$(basename $(dirname $lib))
    TSM_EXPERIMENT_LIB=$lib timeout -k 10 120 python3 tools/remap_probe.py $n 2>&1 | grep form || exit 1
  done
done
