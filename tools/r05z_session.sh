set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r05z_parity.log 2>&1; rc=$?; tail -2 gpurun_out/r05z_parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for x in default nopipe; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  timeout -k 10 200 python3 tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 32 --concurrency 16 --label $x 2>&1 | grep -v "^\[\|WARNING" | tail -1 || exit 1
  timeout -k 10 200 python3 tools/stage_probe.py --pairs 128 --concurrency 64 --single 5 --label $x 2>&1 | grep -v "^\[\|WARNING" | tail -1 || exit 1
  timeout -k 10 200 python3 tools/stage_probe.py --hsi --pairs 64 --concurrency 64 --label $x 2>&1 | grep -v "^\[\|WARNING" | tail -1 || exit 1
done
done
