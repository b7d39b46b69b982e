#!/bin/bash
# GPU box: for the default library and each experiment build (build/exp/<name>), one short
# bench run: pairs/s, one-pipeline stage times and the cost launch's average duration.
#   usage: exp_stage.sh <exp name> ...   (experiment builds are timing probes: outputs unchecked)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for x in default "$@"; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ops --no-configs > gpurun_out/es_$x.log 2>&1 || { echo "$x rc=$?"; tail -5 gpurun_out/es_$x.log; exit 1; }
  python3 - "$x" gpurun_out/es_$x.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], d["value"], d["stage_ms_per_pair"], "cost_launch_ms", d["roofline"]["avg_launch_ms"])
PY
done
