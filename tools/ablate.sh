#!/bin/bash
# GPU box: pairs/s of the bench with stages skipped (experiment build -DTSM_EXP_SKIP,
# results are garbage; timing only) and at several pipeline concurrencies.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TSM_LIB=build/exp/skip/libtsm_adcensus.so
run() {  # run <label> <env...> -- <bench args>
    local label=$1; shift
    env "$@" timeout -k 10 120 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline $BARGS > gpurun_out/ab_$label.log 2>&1
    local rc=$?
    [ $rc -ne 0 ] && { echo "$label rc=$rc"; tail -5 gpurun_out/ab_$label.log; exit $rc; }
    echo "$label $(grep -o '"value": [0-9.]*' gpurun_out/ab_$label.log) $(grep -o '"stage_ms_per_pair": {[^}]*}' gpurun_out/ab_$label.log)"
}
BARGS=""
for s in 0 1 2 3 4 8 16 7 15; do run skip$s TSM_SKIP=$s; done
for c in 1 2 4; do BARGS="--concurrency $c"; run conc$c TSM_SKIP=0; done
