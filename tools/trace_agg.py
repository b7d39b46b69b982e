#!/usr/bin/env python3
"""Per-launch durations of the aggregation / scanline / cost kernels from a rocprofv3 kernel trace."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
acc = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    key = n.split("(")[0][:60] + f" grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}"
    acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:80s} n={len(v):4d} avg_us={sum(v)/len(v):8.1f} min={min(v):8.1f} total_ms={sum(v)/1e3:7.2f}")
