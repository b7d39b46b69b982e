#!/usr/bin/env python3
"""HBM bytes per cost-volume launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
separate passes, kernel filter $KREGEX), with the gfx950 correction of the
microarchitecture guide: FETCH_SIZE counts 64 B per 128-B request of a wide coalesced
read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Both
are in KiB.  Usage: pmc_cost_json.py FETCH.csv WRITE.csv OUT.json [kernel]"""
import collections
import csv
import json
import sys


def per_dispatch(path, counter):
    disp = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            disp[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(disp.values())


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
f_kib = sum(fetch) / len(fetch)
w_kib = sum(write) / len(write)
out = {
    "kernel": (sys.argv[4] if len(sys.argv) > 4 else "k_cost_walk<3,false,false,0>") + " (config B: 1242x375, L=193, both views, one launch)",
    "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
    "fetch_size_kib_raw": f_kib,
    "write_size_kib": w_kib,
    "fetch_bytes_corrected": 2 * f_kib * 1024,
    "write_bytes": w_kib * 1024,
    "hbm_bytes_per_launch": 2 * f_kib * 1024 + w_kib * 1024,
    "algorithmic_bytes_per_launch": 4 * 193 * 1242 * 375 * 2 + 2 * 3 * 1242 * 375,
    "note": "FETCH_SIZE doubled (gfx950: 64 B tallied per 128-B request); Infinity-Cache hits are counted by these fabric-side counters",
}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))
