#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: per-kernel calls, avg, total, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{r['Name'][:58]:58s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:9.1f} "
          f"total_ms={float(r['TotalDurationNs'])/1e6:8.2f} {100*float(r['TotalDurationNs'])/tot:5.1f}%")
