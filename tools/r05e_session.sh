set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05e || exit 1
bash tools/kernel_stats.sh r05e_areal1 tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 1 --concurrency 1 --single 10 || exit 1
for wl in "--png 0600-Left.png 0600-Right.png --pairs 32 --concurrency 16 --single 5" "--pairs 128 --concurrency 64 --single 5" "--png Motorcycle_Left.png Motorcycle_Right.png --max-disparity 256 --pairs 16 --concurrency 8 --single 3"; do
  timeout -k 10 200 python3 tools/stage_probe.py $wl 2>&1 | grep -v "^\[" | tail -1 || exit 1
done
