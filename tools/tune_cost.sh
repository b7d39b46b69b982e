#!/bin/bash
# Runs on the GPU box: cost-walk segment length sweep (stage timing at concurrency 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in "$@"; do
    TSM_COST_SEG=$s timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --concurrency 1 > gpurun_out/tune_$s.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "seg $s rc=$rc"; tail -5 gpurun_out/tune_$s.log; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/tune_$s.log').read().strip().splitlines()[-1]); print('seg', $s, 'value', d['value'], 'stages', d['stage_ms_per_pair'])"
done
