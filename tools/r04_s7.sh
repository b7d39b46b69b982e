#!/bin/bash
# GPU box, round-4 session 7: timing probes of the round-4 streamer (outputs unchecked).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/exp_stage.sh nostore win1 noload noio
