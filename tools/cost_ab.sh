#!/bin/bash
# GPU box: cost-walk timing A/B (kernel trace, concurrency 1): shear (default), shear
# without view-1 stores (timing only), both views walked, and unit lengths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c_$n -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 2 > gpurun_out/c_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/c_$n.log; exit 1; }
  echo "$n: $(python3 tools/trace_agg.py gpurun_out/c_$n/run_kernel_trace.csv | grep -E 'cost_walk|shear_tail' | awk '{print $1, $2, $5, $6}' | tr '\n' ' ')"
}
run shear48 TSM_COST_SEG=48
run shear24 TSM_COST_SEG=24
run shear32 TSM_COST_SEG=32
run noshear TSM_COST_SHEAR=0
run ns1 TSM_LIB=build/exp/ns1/libtsm_adcensus.so
