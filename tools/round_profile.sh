#!/bin/bash
# GPU box: GPU tests, the default bench line, and a rocprofv3 kernel trace + stats of a
# shorter bench run (same configuration), for profiles/<tag>_*.  usage: round_profile.sh <tag>
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TAG=$1
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/${TAG}_tests.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/${TAG}_tests.log; exit $rc; }
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_bench.log; exit $rc; }
grep '^{' gpurun_out/${TAG}_bench.log | tail -1 > gpurun_out/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_prof.log; exit $rc; }
python3 tools/roofline_trace.py gpurun_out/${TAG}_prof/run_kernel_trace.csv 128 > gpurun_out/${TAG}_cost_roofline_trace.json
cat gpurun_out/${TAG}_bench.json
