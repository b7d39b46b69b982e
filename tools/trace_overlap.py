#!/usr/bin/env python3
"""Wall-time attribution over a rocprofv3 kernel trace: over the last `--window` fraction
of the run (the timed region), each instant is split evenly among the kernels running
then, so the shares add up to the wall time; also reports how many kernels co-run."""
import collections
import csv
import sys


def short(n):
    n = n.split("(")[0]
    for p in ("void ", "tsm::"):
        n = n.replace(p, "")
    return n[:48]


rows = list(csv.DictReader(open(sys.argv[1])))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
t_end = max(e for _, e, _ in iv)
t_beg = min(s for s, _, _ in iv)
t0 = t_end - frac * (t_end - t_beg)
ev = []
for s, e, n in iv:
    s, e = max(s, t0), e
    if e <= s:
        continue
    ev.append((s, 1, n))
    ev.append((e, -1, n))
ev.sort()
run = collections.Counter()
share = collections.Counter()
conc = collections.Counter()
last = t0
for t, d, n in ev:
    k = sum(run.values())
    if k and t > last:
        for m, c in run.items():
            share[m] += (t - last) * c / k
        conc[k] += t - last
    elif t > last:
        conc[0] += t - last
    last = t
    run[n] += d
    if run[n] == 0:
        del run[n]
wall = t_end - t0
print(f"window {wall/1e6:.2f} ms")
for m, v in share.most_common(25):
    print(f"{m:50s} {v/1e6:8.3f} ms {100*v/wall:5.1f}%")
print("co-running kernels:", {k: round(100 * v / wall, 1) for k, v in sorted(conc.items())})
