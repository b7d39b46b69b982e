#!/bin/bash
# Runs on the GPU box: default-concurrency bench of experimental library builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for x in "$@"; do
    lib=build/exp/$x/libtsm_adcensus.so; [ "$x" = base ] && lib=tea_stereo_matching_amd/lib/libtsm_adcensus.so
    TSM_LIB=$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abf_$x.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$x rc=$rc"; tail -5 gpurun_out/abf_$x.log; exit $rc; fi
    python3 -c "import json; d=json.loads(open('gpurun_out/abf_$x.log').read().strip().splitlines()[-1]); print('$x full', d['value'])"
done
