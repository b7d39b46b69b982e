#!/usr/bin/env python3
"""HBM bytes per launch of every cost / aggregation / scanline kernel of one config-B pair,
from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs of tools/pmc.sh
with KREGEX="k_agg|k_scan_line|k_cost_walk|k_wta").  gfx950 correction as in
pmc_cost_json.py: FETCH_SIZE doubled, WRITE_SIZE as counted; both in KiB.
Usage: pmc_pipe_json.py FETCH.csv WRITE.csv OUT.json"""
import collections
import csv
import json
import sys

N, L, Lp = 1242 * 375, 193, 196
VOL = 4 * Lp * N * 2  # both views' fp32 label vectors, bytes


def per_kernel(path, counter):
    disp = collections.defaultdict(float)
    name = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            disp[r["Dispatch_Id"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    k = collections.defaultdict(list)
    for d, v in disp.items():
        k[name[d]].append(v)
    return {n: sum(v) / len(v) for n, v in k.items()}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
out = {"config": "B: 1242x375, L=193 (Lp=196), both views", "volume_bytes_both_views": VOL,
       "note": "per launch; FETCH_SIZE doubled (gfx950: 64 B tallied per 128-B request); "
               "fabric-side counters (Infinity-Cache hits included)", "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    f = 2 * fetch.get(k, 0) * 1024
    w = write.get(k, 0) * 1024
    out["kernels"][k] = {"fetch_bytes": round(f), "write_bytes": round(w),
                         "hbm_bytes": round(f + w), "in_volumes": round((f + w) / VOL, 3)}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
