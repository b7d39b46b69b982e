set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TAG=r05o_costB bash tools/pmc_kernel.sh "k_cost_walk" tools/stage_probe.py --pairs 2 --concurrency 1 || exit 1
TAG=r05o_costC bash tools/pmc_kernel.sh "k_cost_walk" tools/stage_probe.py --height 1000 --width 1500 --max-disparity 256 --pairs 2 --concurrency 1 || exit 1
