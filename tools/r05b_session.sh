set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stereo_ops.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05b_ops.log 2>&1
rc=$?; echo "ops tests rc=$rc: $(tail -1 gpurun_out/r05b_ops.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r05b_ops.log; exit $rc; }
bash tools/kernel_stats.sh r05b_areal tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 4 --concurrency 4 --single 5 || exit 1
bash tools/kernel_stats.sh r05b_b tools/stage_probe.py --pairs 4 --concurrency 4 --single 5 || exit 1
TAG=r05b_aggA bash tools/pmc_kernel.sh "k_agg_split" tools/stage_probe.py --png 0600-Left.png 0600-Right.png --pairs 2 --concurrency 1 || exit 1
