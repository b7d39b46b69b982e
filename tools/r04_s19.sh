#!/bin/bash
# GPU box, round-4 final tree after the refine / arms load batching: smoke + GPU suite +
# default bench line (r04_check.sh), and a rocprofv3 kernel trace + stats of a shorter bench.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
T=${1:-r04_v4}
bash tools/r04_check.sh $T || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${T}_prof.log; exit $rc; }
python3 tools/roofline_trace.py gpurun_out/${T}_prof/run_kernel_trace.csv 128 > gpurun_out/${T}_cost_roofline_trace.json || exit 1
python3 tools/trace_share.py gpurun_out/${T}_prof/run_kernel_trace.csv > gpurun_out/${T}_trace_share.txt || exit 1
cp gpurun_out/${T}_prof/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv
cat gpurun_out/${T}_cost_roofline_trace.json
