set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r05k_tests.log 2>&1; rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r05k_tests.log)"; [ $rc -ne 0 ] && exit 1
for x in default colwalk; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  echo "== $x B"; bash tools/kernel_stats.sh r05k_b_$x tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "vote|vprefix|hv_|oscan" || exit 1
  echo "== $x A"; bash tools/kernel_stats.sh r05k_a_$x tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 1 --concurrency 1 --single 10 | grep -E "vote|vprefix" || exit 1
done
