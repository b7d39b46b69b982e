#!/bin/bash
# GPU box: aggregation probes -- stamp split of the v3 streamer, per-launch traces of v3 / v4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
TSM_LIB=build/exp/stamps/libtsm_adcensus.so timeout -k 10 200 python3 tools/agg_stamps.py > gpurun_out/stamps.log 2>&1 || { echo stamps failed; tail gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
for k in dma grp; do
  TSM_AGG_KERNEL=$k timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$k -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --concurrency 1 --batch 2 > gpurun_out/tr_$k.log 2>&1 || { echo trace $k failed; tail gpurun_out/tr_$k.log; exit 1; }
  tail -1 gpurun_out/tr_$k.log | cut -c1-600
done
