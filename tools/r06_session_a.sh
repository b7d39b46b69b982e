bash tools/gpu_suite.sh r06a || exit 1
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r06a_bench.log 2>&1; echo bench rc=$?
tail -c 3000 gpurun_out/r06a_bench.log
EXP_WL="--png 0600-Left.png 0600-Right.png --pairs 32 --concurrency 16" bash tools/exp_probe.sh 2 agg_len20 agg_len1 2>&1 | tee gpurun_out/r06a_probe.txt
