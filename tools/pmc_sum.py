#!/usr/bin/env python3
"""Average per-dispatch value of every counter in rocprofv3 counter_collection CSVs."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        disp[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"][:60]
    kern = collections.defaultdict(list)
    for d, c in disp.items():
        kern[names[d]].append(c)
    for k, lst in kern.items():
        print(f"{path}: {k} ({len(lst)} dispatches)")
        for cn in lst[0]:
            print(f"    {cn:40s} {sum(x[cn] for x in lst) / len(lst):.6g}")
