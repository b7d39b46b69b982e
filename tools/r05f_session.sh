set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05f || exit 1
bash tools/kernel_stats.sh r05f_b1 tools/stage_probe.py --pairs 1 --concurrency 1 --single 10 | grep -E "vote|hv_|oscan|vprefix|rc=" || exit 1
bash tools/exp_probe.sh 1 vk16 plainst
