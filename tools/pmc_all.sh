#!/bin/bash
# GPU box: FETCH_SIZE and WRITE_SIZE (separate passes) of every volume kernel over a short
# bench of single-pair groups (config B) -> gpurun_out/<tag>_pmc_all.json via tools/pmc_all.py.
# usage: pmc_all.sh <tag>
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TAG=${1:-r04}
RX="k_agg_split|k_agg_stream|k_scan_line|k_cost_walk"
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ops --no-configs --batch 2 --concurrency 1"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${TAG}_pmcf -o run -- $B > gpurun_out/${TAG}_pmcf.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_pmcf.log; exit $rc; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${TAG}_pmcw -o run -- $B > gpurun_out/${TAG}_pmcw.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_pmcw.log; exit $rc; }
python3 tools/pmc_all.py gpurun_out/${TAG}_pmcf/run_counter_collection.csv gpurun_out/${TAG}_pmcw/run_counter_collection.csv > gpurun_out/${TAG}_pmc_all.json
cat gpurun_out/${TAG}_pmc_all.json
