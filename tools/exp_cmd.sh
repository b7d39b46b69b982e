set -u
cd "${GRAFT_REPO_ROOT}"
TSM_LIB=build/exp/sh4/libtsm_adcensus.so timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/sh4_tests.log 2>&1
echo "sh4 tests rc=$?: $(tail -1 gpurun_out/sh4_tests.log)"
bash tools/lat_prof_exp.sh sh4 sh4nobar
bash tools/exp_stage.sh elane
