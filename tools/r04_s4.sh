#!/bin/bash
# GPU box, round-4 session 4: stage timings of the split streamer for every pass (+ streaming
# loads on the single passes) against the default, two rounds each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/exp_stage.sh v6all r04base && bash tools/exp_stage.sh v6all
