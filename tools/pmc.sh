#!/bin/bash
# Runs on the GPU box: one rocprofv3 --pmc pass per argument group for kernels matching
# $KREGEX, over a short bench run (concurrency 1).  Usage: KREGEX=cost_walk pmc.sh "A B C" "D E"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
root=$PWD
n=0
for grp in "$@"; do
    n=$((n+1))
    cd /tmp && export TMPDIR=/tmp && cd "$root"
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$KREGEX" --output-format csv \
        -d gpurun_out/pmc_$n -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 2 --concurrency 1 > gpurun_out/pmc_$n.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pass $n rc=$rc"; tail -5 gpurun_out/pmc_$n.log; exit $rc; fi
done
python3 tools/pmc_sum.py gpurun_out/pmc_*/run_counter_collection.csv
