#!/bin/bash
# GPU box: rocprofv3 kernel trace + per-kernel stats of one command (measurement tooling).
#   tools/kernel_stats.sh <tag> <python args...>   e.g.  tools/kernel_stats.sh a_real tools/stage_probe.py --png ...
# -> gpurun_out/<tag>_ks/ (trace + stats csv) and gpurun_out/<tag>_ks.txt (stats summary)
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ks -o run -- python3 "$@" > gpurun_out/${TAG}_ks.log 2>&1
rc=$?; echo "$TAG rc=$rc: $(grep -v '^\[' gpurun_out/${TAG}_ks.log | tail -1)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_ks.log; exit $rc; }
f=$(ls gpurun_out/${TAG}_ks/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:25]:
    print(f\"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} calls {float(r['AverageNs'])/1e3:9.2f} us avg {100*float(r['TotalDurationNs'])/tot:5.1f}%  {r['Name'][:90]}\")
" > gpurun_out/${TAG}_ks.txt
cat gpurun_out/${TAG}_ks.txt
