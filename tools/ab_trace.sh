#!/bin/bash
# GPU box: per-launch kernel traces (concurrency 1) of experimental library builds.
#   ab_trace.sh [--test] name...   (name "base" = the in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
test=0; [ "${1:-}" = "--test" ] && { test=1; shift; }
for x in "$@"; do
  lib=build/exp/$x/libtsm_adcensus.so; [ "$x" = base ] && lib=tea_stereo_matching_amd/lib/libtsm_adcensus.so
  if [ $test = 1 ]; then
    TSM_EXPERIMENT_LIB=$lib timeout -k 10 300 python3 -m pytest tests -x -q -m gpu > gpurun_out/abt_test_$x.log 2>&1
    rc=$?; echo "$x tests rc=$rc: $(tail -1 gpurun_out/abt_test_$x.log)"; [ $rc -gt 1 ] && exit $rc
  fi
  TSM_EXPERIMENT_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abt_$x -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 2 > gpurun_out/abt_$x.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$x rc=$rc"; tail -5 gpurun_out/abt_$x.log; exit $rc; }
  echo "== $x"; python3 tools/trace_agg.py gpurun_out/abt_$x/run_kernel_trace.csv | head -${TOPN:-8}
done
