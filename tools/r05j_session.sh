set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for x in default hk32; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  echo "== $x"; bash tools/kernel_stats.sh r05j_$x tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "k_scan_line<1, (16|32), true" || exit 1
done
