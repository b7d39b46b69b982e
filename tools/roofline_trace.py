#!/usr/bin/env python3
"""Average duration of the cost-volume launches of bench.py's roofline phase, from a
rocprofv3 --kernel-trace CSV of the same bench command.

bench.py runs its timed region with two pipelines (kernels co-run, groups of 64 pairs),
then the roofline phase: the batch again through ONE pipeline in groups of one, whose
`batch` cost-walk dispatches (grid z = 1, the headline kernel) run alone; the configs leg's
single-pair launches come after them.  Their rocprof average is the number that must agree
with the bench line's roofline.avg_launch_ms (HIP events).  Usage: roofline_trace.py run_kernel_trace.csv [batch]
"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_cost_walk" in r["Kernel_Name"] or "k_cost_mfma" in r["Kernel_Name"]]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the headline kernel is the one of the first group launch (grid z > 1); the roofline phase
# ends the longest run of its single-pair launches (grid z = 1: the host leg's single frames,
# then the phase); the configs leg's single-pair runs are shorter
main = [r for r in rows if r.get("Grid_Size_Z") != "1"]
head = main[0]["Kernel_Name"] if main else (rows[0]["Kernel_Name"] if rows else "")
runs, cur = [], []
for r in rows:
    if r["Kernel_Name"] == head and r.get("Grid_Size_Z") == "1":
        cur.append(r)
    elif cur:
        runs.append(cur)
        cur = []
if cur:
    runs.append(cur)
run = max(runs, key=len) if runs else []
last = run[-batch:] if run else rows[-batch:]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in last]
print(json.dumps({
    "kernel": last[0]["Kernel_Name"] if last else None,
    "roofline_phase_dispatches": len(d),
    "avg_us": round(sum(d) / max(1, len(d)), 2),
    "min_us": round(min(d), 2) if d else None,
    "max_us": round(max(d), 2) if d else None,
    "all_dispatches": len(rows),
    "all_avg_us": round(sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows) / max(1, len(rows)), 2),
}, indent=1))
