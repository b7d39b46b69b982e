set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for x in default st4 nost; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  echo "== $x B"; bash tools/kernel_stats.sh r05u_b_$x tools/stage_probe.py --pairs 64 --concurrency 64 | grep -E "k_cost|rc=" || exit 1
  echo "== $x B1"; bash tools/kernel_stats.sh r05u_b1_$x tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "k_cost|rc=" || exit 1
done
