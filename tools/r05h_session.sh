set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05h || exit 1
bash tools/kernel_stats.sh r05h_b1 tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "vote|rc=" || exit 1
bash tools/kernel_stats.sh r05h_a1 tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 1 --concurrency 1 --single 10 | grep -E "vote|rc=" || exit 1
for wl in "--png 0600-Left.png 0600-Right.png --pairs 32 --concurrency 16 --single 5" "--pairs 128 --concurrency 64 --single 5"; do
  timeout -k 10 200 python3 tools/stage_probe.py $wl 2>&1 | grep -v "^\[" | tail -1 || exit 1
done
bash tools/pmc_all.sh r05h_C 1000 1500 257 "config C (synthetic)" -- --height 1000 --width 1500 --max-disparity 256 || exit 1
bash tools/pmc_all.sh r05h_E 1536 2048 321 "config E (synthetic grey)" -- --height 1536 --width 2048 --max-disparity 320 --grey || exit 1
bash tools/pmc_all.sh r05h_A 720 1280 193 "A_real (demo-imgs/0600)" -- --png 0600-Left.png 0600-Right.png || exit 1
