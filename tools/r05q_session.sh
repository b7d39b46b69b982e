set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05q || exit 1
for x in default unpipe pipew4; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  echo "== $x B"; bash tools/kernel_stats.sh r05q_b_$x tools/stage_probe.py --pairs 64 --concurrency 64 | grep -E "k_cost_walk|rc=" || exit 1
  echo "== $x C"; bash tools/kernel_stats.sh r05q_c_$x tools/stage_probe.py --height 1000 --width 1500 --max-disparity 256 --pairs 8 --concurrency 8 | grep -E "k_cost_walk|rc=" || exit 1
  echo "== $x A"; bash tools/kernel_stats.sh r05q_a_$x tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 16 --concurrency 16 | grep -E "k_cost_walk|rc=" || exit 1
done
