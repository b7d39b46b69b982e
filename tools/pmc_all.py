#!/usr/bin/env python3
"""Per-kernel HBM bytes per dispatch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
single-pair launches, against each kernel's algorithmic bytes.
FETCH_SIZE is doubled (gfx950 tallies 64 B per 128-B request, MI355X_MICROARCH.md).

    pmc_all.py fetch.csv write.csv [H W L label]      (default: config B, 375 1242 193)"""
import collections
import csv
import json
import sys

H, W, L = (int(x) for x in sys.argv[3:6]) if len(sys.argv) >= 6 else (375, 1242, 193)
LABEL = sys.argv[6] if len(sys.argv) >= 7 else "config B (synthetic)"
LP = (L + 3) // 4 * 4
N = H * W
VOL = 2 * LP * N * 4  # the two-view volume at the padded stride, one pair


def per(path, counter):
    d = collections.defaultdict(float)
    name = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[r["Dispatch_Id"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = r["Kernel_Name"]
    k = collections.defaultdict(list)
    for i, v in d.items():
        k[name[i]].append(v * 1024)  # rocprofv3 reports KiB
    return k


def short(n):
    return n.split("(")[0].replace("void ", "").replace("tsm::", "")


def algorithmic(n):
    if "k_cost_walk" in n:
        return 4 * L * N * 2 + 2 * 3 * N, "B_build (write both views + images)"
    if "k_agg" in n:
        return 2 * VOL, "read + write of the two-view volume"
    if "k_scan_line" in n and "true, true" in n.split(">")[0]:
        return 1.5 * VOL, "leftward + WTA: read both views, write view 0"
    if "k_scan_line" in n:
        return 2 * VOL, "read + write of the two-view volume"
    return None, None


f, w = per(sys.argv[1], "FETCH_SIZE"), per(sys.argv[2], "WRITE_SIZE")
out = {"note": f"bytes per dispatch; FETCH_SIZE x2 (gfx950); single-pair launches of {LABEL} "
               f"({W}x{H}, {L} labels); a scanline pass leaves a pixel untouched when its predecessor's "
               "minimum is exactly 0 (ADCensus.cpp:880-881) and then does not store it: exact-shift "
               "synthetic pairs have many such pixels, noisy and real pairs none, so on synthetic pairs "
               "the scanline's write is below the algorithmic bound",
       "workload": {"H": H, "W": W, "L": L, "label": LABEL},
       "kernels": {}}
for n in sorted(set(f) | set(w)):
    fb = 2 * sum(f[n]) / len(f[n]) if f.get(n) else None
    wb = sum(w[n]) / len(w[n]) if w.get(n) else None
    alg, what = algorithmic(n)
    e = {"dispatches": [len(f.get(n, [])), len(w.get(n, []))], "fetch_bytes": fb, "write_bytes": wb,
         "algorithmic_bytes": alg, "algorithmic": what}
    if alg and fb is not None and wb is not None:
        e["ratio"] = round((fb + wb) / alg, 4)
    out["kernels"][short(n)] = e
print(json.dumps(out, indent=1))
