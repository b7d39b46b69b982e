#!/usr/bin/env python3
"""Average duration of the cost-volume launches of bench.py's roofline phase, from a
rocprofv3 --kernel-trace CSV of the same bench command.

bench.py runs its timed region with two pipelines (kernels co-run), then the roofline
phase: the batch again through ONE pipeline, so the last `batch` cost-walk dispatches run
alone.  Their rocprof average is the number that must agree with the bench line's
roofline.avg_launch_ms (HIP events).  Usage: roofline_trace.py run_kernel_trace.csv [batch]
"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_cost_walk" in r["Kernel_Name"] or "k_cost_mfma" in r["Kernel_Name"]]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-batch:]
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
