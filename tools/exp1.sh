set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/stream_hbm.py > gpurun_out/e1_stream.log 2>&1 || exit $?
cat gpurun_out/e1_stream.log
for lib in default w1; do
  if [ $lib = default ]; then unset TSM_LIB; else export TSM_LIB=build/exp/$lib/libtsm_adcensus.so; fi
  timeout -k 10 120 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 4 > gpurun_out/e1_$lib.log 2>&1 || exit $?
  echo "$lib $(grep -o '"value": [0-9.]*' gpurun_out/e1_$lib.log) $(grep -o '"stage_ms_per_pair": {[^}]*}' gpurun_out/e1_$lib.log)"
done
