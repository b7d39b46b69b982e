#!/bin/bash
# GPU box: smoke, the GPU suite (-v), then the default bench line.  usage: r04_check.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/${TAG}_smoke.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python3 -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | grep -v PASSED | head -40
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_bench.log; exit $rc; }
grep '^{' gpurun_out/${TAG}_bench.log | tail -1 > gpurun_out/${TAG}_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json'))
print('value', d['value'], 'verified', d['verified'], 'frac', d['roofline']['frac'], 'host', d.get('host_buffers'))
for k,v in (d.get('configs') or {}).items():
    print(k, v if isinstance(v,str) else {x: v[x] for x in ('pairs_per_s','ms_per_frame','single_frame_device_ms','verified')}, '' if isinstance(v,str) else v['cost_walk']['frac'])
print('cpu', d.get('cpu_baseline'))
"
