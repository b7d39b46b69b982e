#!/bin/bash
# GPU box: cost-walk timing A/B (kernel trace, concurrency 1): current default, E = 4,
# per-view launches, segment lengths, shear.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c_$n -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 2 > gpurun_out/c_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/c_$n.log; exit 1; }
  echo "$n: $(python3 tools/trace_agg.py gpurun_out/c_$n/run_kernel_trace.csv | grep -E 'cost_walk|shear_tail' | sed 's/  */ /g' | cut -c1-150 | tr '\n' '|')"
}
for a in "$@"; do
  case $a in
    cur) run cur TSM_COST_SEG=48 ;;
    e4) run e4 TSM_COST_E4=1 ;;
    views) run views TSM_COST_VIEWS=1 ;;
    e4views) run e4views TSM_COST_VIEWS=1 TSM_COST_E4=1 ;;
    views32) run views32 TSM_COST_SEG=32 ;;
    seg72) run seg72 TSM_COST_SEG=72 ;;
    seg96) run seg96 TSM_COST_SEG=96 ;;
    seg144) run seg144 TSM_COST_SEG=144 ;;
    views64) run views64 TSM_COST_SEG=64 ;;
    both) run both TSM_COST_BOTH=1 ;;
    shear) run shear TSM_COST_SHEAR=1 ;;
  esac
done
