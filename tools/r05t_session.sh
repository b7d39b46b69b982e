set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05t || exit 1
echo "== B"; bash tools/kernel_stats.sh r05t_b tools/stage_probe.py --pairs 64 --concurrency 64 | grep -E "k_cost|rc=" || exit 1
echo "== A"; bash tools/kernel_stats.sh r05t_a tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 16 --concurrency 16 | grep -E "k_cost|rc=" || exit 1
echo "== B1"; bash tools/kernel_stats.sh r05t_b1 tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "k_cost|rc=" || exit 1
