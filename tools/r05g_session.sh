set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05g || exit 1
bash tools/kernel_stats.sh r05g_b1 tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "vote|rc=" || exit 1
EXP_WL="--png 0600-Left.png 0600-Right.png --pairs 32 --concurrency 16 --single 5" bash tools/exp_probe.sh 2 aggprio
TAG=r05g_aggA bash tools/pmc_kernel.sh "k_agg_split" tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 2 --concurrency 1 || exit 1
