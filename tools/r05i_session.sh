set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05i || exit 1
bash tools/kernel_stats.sh r05i_b1 tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "vote|vpre|oscan|hv_|rc=" || exit 1
bash tools/kernel_stats.sh r05i_a1 tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 1 --concurrency 1 --single 10 | grep -E "vote|vpre|oscan|hv_|rc=" || exit 1
for wl in "--png 0600-Left.png 0600-Right.png --pairs 32 --concurrency 16 --single 5" "--pairs 128 --concurrency 64 --single 5"; do
  timeout -k 10 200 python3 tools/stage_probe.py $wl 2>&1 | grep -v "^\[" | tail -1 || exit 1
done
for x in default hnowmin hnostore; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  echo "== $x"; bash tools/kernel_stats.sh r05i_$x tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "k_scan_line<1, 16, true" || exit 1
done
