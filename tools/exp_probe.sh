#!/bin/bash
# GPU box: same-box A/B of experiment builds (build/exp/<name>) against the default library
# over tools/stage_probe.py workloads (real 0600 pair, config B, config B noisy, HSI, Moto).
#   usage: exp_probe.sh <reps> <exp name> ...      (timing probes: outputs unchecked)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=$1; shift
WL=("--png 0600-Left.png 0600-Right.png --pairs 32 --concurrency 16 --single 5"
    "--pairs 128 --concurrency 64 --single 5"
    "--noisy --pairs 128 --concurrency 64 --single 5")
[ -n "${EXP_WL:-}" ] && WL=("$EXP_WL")
for r in $(seq $REPS); do
  for wl in "${WL[@]}"; do
    for x in default "$@"; do
      if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
      timeout -k 10 200 python3 tools/stage_probe.py $wl --label $x 2>&1 | grep -v "^\[\|WARNING" | tail -1 || exit 1
    done
  done
done
