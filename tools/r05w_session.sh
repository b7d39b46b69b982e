set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for r in 1 2; do
for x in default ringoff; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  echo "== $x B1 $r"; bash tools/kernel_stats.sh r05w_b1_${x}_$r tools/stage_probe.py --pairs 1 --concurrency 1 --single 20 | grep -E "k_cost|rc=" || exit 1
  echo "== $x B $r"; bash tools/kernel_stats.sh r05w_b_${x}_$r tools/stage_probe.py --pairs 64 --concurrency 64 | grep -E "k_cost|rc=" || exit 1
done
done
