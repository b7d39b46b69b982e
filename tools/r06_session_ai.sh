#!/bin/bash
# round-6 session ai: bench with the second-handle repeat -- contract test, the default bench
# line, the two-rank rehearsal
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bench_contract.py -x -q --timeout 280 --timeout-method thread > gpurun_out/ai_contract.log 2>&1
rc=$?; echo "contract rc=$rc: $(tail -1 gpurun_out/ai_contract.log)"; [ $rc -ne 0 ] && { tail -20 gpurun_out/ai_contract.log; exit $rc; }
timeout -k 10 600 python3 bench.py > gpurun_out/ai_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/ai_bench.log; exit $rc; }
grep '^{' gpurun_out/ai_bench.log | tail -1 > gpurun_out/ai_bench.json
python3 -c "import json;d=json.load(open('gpurun_out/ai_bench.json'));print(d['value'], json.dumps(d['timed_region']), d['configs']['B_OMP20']['pairs_per_s'])"
bash tools/rehearse_n2.sh
