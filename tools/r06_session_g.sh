#!/bin/bash
# round-6 session g: cost walk stores on config C (nt vs plain), config E aggregation PMC on the
# current tree, SQ counters of the HSI cost walk
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
CARGS="--height 1000 --width 1500 --max-disparity 256"
for x in default cost_e4_plain default cost_e4_plain; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  timeout -k 10 200 python3 tools/stage_probe.py $CARGS --pairs 8 --concurrency 4 --label $x 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee -a gpurun_out/r06g_c_stage.txt || exit 1
done
unset TSM_EXPERIMENT_LIB
bash tools/pmc_all.sh r06g_C 1000 1500 257 "config C (synthetic)" -- $CARGS || exit 1
export TSM_EXPERIMENT_LIB=build/exp/cost_e4_plain/libtsm_adcensus.so
bash tools/pmc_all.sh r06g_Cplain 1000 1500 257 "config C (synthetic), plain cost stores" -- $CARGS || exit 1
unset TSM_EXPERIMENT_LIB
bash tools/pmc_all.sh r06g_E 1536 2048 321 "config E (synthetic grey)" -- --height 1536 --width 2048 --max-disparity 320 --grey || exit 1
TAG=r06g_hsi bash tools/pmc_kernel.sh "k_cost_walk" tools/stage_probe.py --hsi --pairs 2 --concurrency 1 > gpurun_out/r06g_hsi_sq.txt 2>&1 || exit 1
tail -30 gpurun_out/r06g_hsi_sq.txt
