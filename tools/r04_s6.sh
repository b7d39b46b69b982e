#!/bin/bash
# GPU box, round-4 session 6: scanline probes (vertical passes with 16 steps in flight;
# streaming loads of the pixel vectors) against the default, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/exp_stage.sh vk16 scannt && bash tools/exp_stage.sh vk16 scannt
