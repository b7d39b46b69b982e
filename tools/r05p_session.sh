set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05p || exit 1
bash tools/kernel_stats.sh r05p_b1 tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "k_scan_line|rc=" || exit 1
for x in default armsb8; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  echo "== $x A"; bash tools/kernel_stats.sh r05p_a_$x tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 1 --concurrency 1 --single 10 | grep -E "k_arms|k_window|k_scan_line<1, 16" || exit 1
  echo "== $x B"; bash tools/kernel_stats.sh r05p_bb_$x tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "k_arms" || exit 1
done
