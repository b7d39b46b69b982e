#!/bin/bash
# GPU box: single-frame latency (tools/latency.py) and a kernel + memory-copy trace of it,
# then the timeline of one device frame and one host frame.  usage: lat_trace.sh <tag>
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TAG=${1:-lat}
timeout -k 10 200 python3 tools/latency.py 1 > gpurun_out/${TAG}_lat.log 2>&1 || { echo "lat rc=$?"; tail gpurun_out/${TAG}_lat.log; exit 1; }
cat gpurun_out/${TAG}_lat.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_trace -o run -- python3 tools/latency.py 1 > gpurun_out/${TAG}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_trace.log; exit $rc; }
K=$(ls gpurun_out/${TAG}_trace/run_kernel_trace.csv gpurun_out/${TAG}_trace/*/run_kernel_trace.csv 2>/dev/null | head -1)
M=$(ls gpurun_out/${TAG}_trace/run_memory_copy_trace.csv gpurun_out/${TAG}_trace/*/run_memory_copy_trace.csv 2>/dev/null | head -1)
python3 tools/frame_timeline.py $K $M --frame=15 > gpurun_out/${TAG}_timeline_host.txt
python3 tools/frame_timeline.py $K $M --frame=40 > gpurun_out/${TAG}_timeline_device.txt
tail -3 gpurun_out/${TAG}_timeline_host.txt gpurun_out/${TAG}_timeline_device.txt
