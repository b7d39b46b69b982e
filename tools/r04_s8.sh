#!/bin/bash
# GPU box, round-4 session 8: cost-walk prologue probe (no wait for the staging / tables).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/exp_stage.sh cwnopro && bash tools/exp_stage.sh cwnopro
