#!/bin/bash
# GPU box, round-4 final tree (continued): the cost walk's HBM bytes and SQ sets
# (pmc_cost.sh), and FETCH/WRITE of every volume kernel (pmc_all.sh).
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
T=r04_v3
bash tools/pmc_cost.sh k_cost_walk > gpurun_out/${T}_pmc_cost.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_cost.log; exit 1; }
cp gpurun_out/cost_pmc.json gpurun_out/${T}_cost_pmc.json
tail -12 gpurun_out/${T}_pmc_cost.log
bash tools/pmc_all.sh $T > gpurun_out/${T}_pmc_all.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_all.log; exit 1; }
cat gpurun_out/${T}_pmc_all.json
