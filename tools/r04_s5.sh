#!/bin/bash
# GPU box, round-4 session 5: smoke + GPU suite + default bench on the single-streamer
# aggregation, then the rocprofv3 kernel trace / stats of a short bench (profiles) and the
# per-kernel PMC bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r04_check.sh r04e || exit $?
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
TAG=r04e
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_prof.log; exit $rc; }
python3 tools/roofline_trace.py gpurun_out/${TAG}_prof/run_kernel_trace.csv 128 > gpurun_out/${TAG}_cost_roofline_trace.json
cp gpurun_out/${TAG}_prof/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
python3 tools/trace_share.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_trace_share.txt 2>&1 || true
cat gpurun_out/${TAG}_cost_roofline_trace.json; head -14 gpurun_out/${TAG}_trace_share.txt
bash tools/pmc_all.sh r04e
