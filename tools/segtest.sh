cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
for sg in 48 96 144; do
  TSM_COST_SEG=$sg timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/seg$sg -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 2 > gpurun_out/seg$sg.log 2>&1 || exit 1
  echo "seg $sg: $(python3 tools/trace_agg.py gpurun_out/seg$sg/run_kernel_trace.csv | grep cost_walk)"
done
