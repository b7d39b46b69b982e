#!/bin/bash
# GPU box: SQ counters of one kernel (regex $1) over a short bench (groups of 2 pairs), or
# over the python command given after the regex; one rocprofv3 --pmc pass per counter set;
# summary by tools/pmc_sum.py.   usage: TAG=x pmc_kernel.sh <regex> [python args...]
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
RX=$1; shift
if [ $# -gt 0 ]; then CMD=("$@"); else
  CMD=(bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ops --no-configs --batch ${PMC_BATCH:-4} --concurrency ${PMC_CONC:-2}); fi
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_SMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pk_${TAG:-x}_$i -o run -- python3 "${CMD[@]}" > gpurun_out/pk_${TAG:-x}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pk_${TAG:-x}_$i.log; exit $rc; }
done
python3 tools/pmc_sum.py gpurun_out/pk_${TAG:-x}_*/run_counter_collection.csv
