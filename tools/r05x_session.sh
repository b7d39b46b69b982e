set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05x || exit 1
for r in 1 2; do
for x in default noshare; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  timeout -k 10 200 python3 tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 32 --concurrency 16 --single 5 --label $x 2>&1 | grep -v "^\[\|WARNING" | tail -1 || exit 1
  timeout -k 10 200 python3 tools/stage_probe.py --pairs 128 --concurrency 64 --single 5 --label $x 2>&1 | grep -v "^\[\|WARNING" | tail -1 || exit 1
  timeout -k 10 200 python3 tools/stage_probe.py --noisy --pairs 128 --concurrency 64 --single 5 --label $x 2>&1 | grep -v "^\[\|WARNING" | tail -1 || exit 1
done
done
