#!/bin/bash
# GPU box, round-4 final tree: smoke + GPU suite + default bench line (r04_check.sh), a
# rocprofv3 kernel trace + stats of a shorter bench, the cost walk's HBM bytes and SQ sets
# (pmc_cost.sh), and FETCH/WRITE of every volume kernel (pmc_all.sh).  Each step under its
# own timeout; the script stops at the first failure.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
T=r04_v3
bash tools/r04_check.sh $T || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${T}_prof.log; exit $rc; }
python3 tools/roofline_trace.py gpurun_out/${T}_prof/run_kernel_trace.csv 128 > gpurun_out/${T}_cost_roofline_trace.json || exit 1
python3 tools/trace_share.py gpurun_out/${T}_prof/run_kernel_trace.csv > gpurun_out/${T}_trace_share.txt || exit 1
cp gpurun_out/${T}_prof/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv
bash tools/pmc_cost.sh k_cost_walk > gpurun_out/${T}_pmc_cost.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_cost.log; exit 1; }
cp gpurun_out/cost_pmc.json gpurun_out/${T}_cost_pmc.json
bash tools/pmc_all.sh $T > gpurun_out/${T}_pmc_all.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_all.log; exit 1; }
echo done
