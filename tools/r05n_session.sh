set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh r05n || exit 1
EXP_WL="--height 1000 --width 1500 --max-disparity 256 --pairs 16 --concurrency 8 --single 3" bash tools/exp_probe.sh 2 slicey
EXP_WL="--png Motorcycle_Left.png Motorcycle_Right.png --max-disparity 256 --pairs 16 --concurrency 8 --single 3" bash tools/exp_probe.sh 1 slicey
bash tools/pmc_all.sh r05n_C 1000 1500 257 "config C (synthetic), slices interleaved" -- --height 1000 --width 1500 --max-disparity 256 || exit 1
