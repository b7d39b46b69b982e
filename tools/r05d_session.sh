set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05d || exit 1
bash tools/kernel_stats.sh r05d_areal1 tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 1 --concurrency 1 --single 10 || exit 1
TAG=r05d_scanA bash tools/pmc_kernel.sh "k_scan_line" tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 2 --concurrency 1 || exit 1
