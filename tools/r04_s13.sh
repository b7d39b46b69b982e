#!/bin/bash
# GPU box, round-4 session 13: the streamer's two-pixels-a-wave form (make exp pw2: masked
# window tails; pw2div: divergent per-lane loops) against the default at config C's and E's
# sizes (timing probes: outputs unchecked; parity of pw2 was checked in session 12).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/s13.txt
run() {  # experiment name, stage_probe args...
  local x=$1; shift
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  timeout -k 10 240 python3 tools/stage_probe.py --label $x "$@" >> gpurun_out/s13.txt 2>&1 || { echo "$x rc=$?"; tail -5 gpurun_out/s13.txt; exit 1; }
  tail -1 gpurun_out/s13.txt
}
for x in default pw2 pw2div; do run $x --height 1000 --width 1500 --max-disparity 256 --pairs 16 --concurrency 8; done
for x in default pw2div; do run $x --height 1536 --width 2048 --max-disparity 320 --pairs 8 --concurrency 4; done
