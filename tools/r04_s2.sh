#!/bin/bash
# GPU box, round-4 session 2: rocprofv3 kernel stats of the default bench (short) + the
# cost-walk roofline-phase trace, then SQ counters of the fused aggregation and the
# vertical scanline in groups of 8 pairs.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TAG=r04b
bash tools/exp_stage.sh nobar nostore win1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_prof.log; exit $rc; }
K=$(ls gpurun_out/${TAG}_prof/run_kernel_trace.csv gpurun_out/${TAG}_prof/*/run_kernel_trace.csv 2>/dev/null | head -1)
S=$(ls gpurun_out/${TAG}_prof/run_kernel_stats.csv gpurun_out/${TAG}_prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/roofline_trace.py $K 128 > gpurun_out/${TAG}_cost_roofline_trace.json
cp $S gpurun_out/${TAG}_kernel_stats.csv
python3 tools/trace_share.py $K > gpurun_out/${TAG}_trace_share.txt 2>&1 || true
grep '^{' gpurun_out/${TAG}_prof.log | tail -1 > gpurun_out/${TAG}_prof_bench.json
cat gpurun_out/${TAG}_cost_roofline_trace.json; head -12 gpurun_out/${TAG}_kernel_stats.csv | cut -c1-160; cat gpurun_out/${TAG}_trace_share.txt | head -30
TAG=agg PMC_BATCH=16 PMC_CONC=8 bash tools/pmc_kernel.sh "k_agg_split" > gpurun_out/r04b_pmc_agg.txt 2>&1; rc=$?; echo "pmc agg rc=$rc"; cat gpurun_out/r04b_pmc_agg.txt | tail -45; [ $rc -ne 0 ] && exit $rc
TAG=scan PMC_BATCH=16 PMC_CONC=8 bash tools/pmc_kernel.sh "k_scan_line<1, 8, false" > gpurun_out/r04b_pmc_scan.txt 2>&1; rc=$?; echo "pmc scan rc=$rc"; cat gpurun_out/r04b_pmc_scan.txt | tail -45
