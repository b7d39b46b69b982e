#!/bin/bash
# Runs on the GPU box: smoke, GPU parity tests, short bench.  Every GPU step has its own
# time limit; a fault / abort / segfault / timeout stops the script (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout-s> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    # 0 ok, 1 test failures (no fault) -> continue; anything else -> stop
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
    return 0
}
for s in "$@"; do
    case $s in
        smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
        trace) export TSM_TRACE=1; step trace 120 python3 -u -c "import __graft_entry__ as g; g.smoke()"; unset TSM_TRACE ;;
        tests) step gpu_tests 900 python3 -m pytest tests -x -q -m gpu ;;
        tests-k) step gpu_tests 900 python3 -m pytest tests -q -m gpu ;;
        bench) step bench 600 python3 bench.py ;;
        bench-short) step bench 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
        prof) cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
              step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
        pmc-fetch) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 2 ;;
        pmc-write) step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 2 ;;
        stream) step stream 300 python3 tools/stream_hbm.py ;;
        pmc-cost-sq) step pmc_cost_sq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS --kernel-include-regex cost_walk --output-format csv -d gpurun_out/pmc_cost_sq -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 2 --concurrency 1 ;;
        pmc-cost-lds) step pmc_cost_lds 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES --kernel-include-regex cost_walk --output-format csv -d gpurun_out/pmc_cost_lds -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 2 --concurrency 1 ;;
        pmc-cost-write) step pmc_cost_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex cost_walk --output-format csv -d gpurun_out/pmc_cost_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 2 --concurrency 1 ;;
        pmc-cost-fetch) step pmc_cost_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex cost_walk --output-format csv -d gpurun_out/pmc_cost_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 2 --concurrency 1 ;;
        pmc-cost) cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
              step pmc_cost_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex cost_walk --output-format csv -d gpurun_out/pmc_cost_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 2 --concurrency 1
              step pmc_cost_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex cost_walk --output-format csv -d gpurun_out/pmc_cost_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 2 --concurrency 1
              python3 tools/pmc_cost_json.py gpurun_out/pmc_cost_fetch/run_counter_collection.csv gpurun_out/pmc_cost_write/run_counter_collection.csv gpurun_out/cost_pmc.json ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
