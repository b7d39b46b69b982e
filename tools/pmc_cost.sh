#!/bin/bash
# GPU box: HBM bytes (FETCH_SIZE, WRITE_SIZE: separate passes) and SQ counters of the cost
# kernel (regex $1, default cost_tile) over a short bench of single-pair groups; summaries
# gpurun_out/cost_pmc.json (tools/pmc_cost_json.py) and tools/pmc_sum.py.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
RX=${1:-cost_tile}
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ops --no-configs --batch 2 --concurrency 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc_cost_fetch -o run -- $B > gpurun_out/pmc_cost_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_cost_fetch.log; exit $rc; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc_cost_write -o run -- $B > gpurun_out/pmc_cost_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_cost_write.log; exit $rc; }
python3 tools/pmc_cost_json.py gpurun_out/pmc_cost_fetch/run_counter_collection.csv gpurun_out/pmc_cost_write/run_counter_collection.csv gpurun_out/cost_pmc.json "$RX"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_SMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pk_$i -o run -- $B > gpurun_out/pk_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pk_$i.log; exit $rc; }
done
python3 tools/pmc_sum.py gpurun_out/pk_*/run_counter_collection.csv
