#!/bin/bash
# GPU box: FETCH_SIZE and WRITE_SIZE (separate passes) of every volume kernel over single-pair
# groups -> gpurun_out/<tag>_pmc_all.json via tools/pmc_all.py.
# usage: pmc_all.sh <tag> [H W L label -- stage_probe args...]   (default: bench.py config B)
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TAG=${1:-r05}; shift || true
RX="k_agg_split|k_scan_line|k_cost_walk"
if [ $# -ge 5 ]; then
  SHAPE=("$1" "$2" "$3" "$4"); shift 5
  B=(python3 tools/stage_probe.py "$@" --pairs 2 --concurrency 1)
else
  SHAPE=(375 1242 193 "config B (synthetic)")
  B=(python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ops --no-configs --batch 2 --concurrency 1)
fi
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${TAG}_pmcf -o run -- "${B[@]}" > gpurun_out/${TAG}_pmcf.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_pmcf.log; exit $rc; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${TAG}_pmcw -o run -- "${B[@]}" > gpurun_out/${TAG}_pmcw.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_pmcw.log; exit $rc; }
python3 tools/pmc_all.py gpurun_out/${TAG}_pmcf/run_counter_collection.csv gpurun_out/${TAG}_pmcw/run_counter_collection.csv "${SHAPE[@]}" > gpurun_out/${TAG}_pmc_all.json
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_pmc_all.json'))
for k,v in d['kernels'].items(): print(f\"{v.get('ratio')}  fetch {v['fetch_bytes']/1e6 if v['fetch_bytes'] else 0:.1f} MB write {v['write_bytes']/1e6 if v['write_bytes'] else 0:.1f} MB alg {v['algorithmic_bytes']/1e6 if v['algorithmic_bytes'] else 0:.1f}  {k}\")"
