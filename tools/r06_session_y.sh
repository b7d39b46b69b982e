#!/bin/bash
# round-6 session y: bench's multi-rank path rehearsed (two gloo ranks on one GPU), cost-walk PMC
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/rehearse_n2.sh || exit 1
bash tools/pmc_cost.sh k_cost_walk > gpurun_out/r06y_pmc_cost.log 2>&1 || { tail -5 gpurun_out/r06y_pmc_cost.log; exit 1; }
cat gpurun_out/cost_pmc.json
