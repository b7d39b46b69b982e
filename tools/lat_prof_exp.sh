#!/bin/bash
# GPU box: kernel trace of tools/latency.py for the default library and experiment builds;
# prints per-kernel medians of the scanline and voting kernels.  usage: lat_prof_exp.sh <exp> ...
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for x in default "$@"; do
  if [ $x = default ]; then unset TSM_EXPERIMENT_LIB; else export TSM_EXPERIMENT_LIB=build/exp/$x/libtsm_adcensus.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lpe_$x -o run -- python3 tools/latency.py 1 > gpurun_out/lpe_$x.log 2>&1 || { echo "$x rc=$?"; tail -5 gpurun_out/lpe_$x.log; exit 1; }
  echo "== $x: $(grep device gpurun_out/lpe_$x.log)"
  python3 - gpurun_out/lpe_$x/run_kernel_trace.csv <<'PY'
import csv, re, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("tsm::", "")
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sorted(kv[1])[len(kv[1]) // 2] * len(kv[1])):
    v.sort()
    if v[len(v) // 2] > 8: print(f"  {k[:60]:60s} n={len(v):4d} med={v[len(v) // 2]:8.1f}")
PY
done
