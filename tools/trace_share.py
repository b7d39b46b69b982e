#!/usr/bin/env python3
"""Effective GPU time per kernel class over a window of a rocprofv3 kernel trace: every
instant is split equally among the kernels active at that instant, so the classes sum to
the window's busy time.  Usage: trace_share.py run_kernel_trace.csv [t_from_ms t_to_ms]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("tsm::", "")
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
t0 = min(e[0] for e in ev)
lo = float(sys.argv[2]) * 1e6 + t0 if len(sys.argv) > 2 else t0
hi = float(sys.argv[3]) * 1e6 + t0 if len(sys.argv) > 3 else max(e[1] for e in ev)
pts = sorted({lo, hi} | {max(lo, min(hi, t)) for s, e, _ in ev for t in (s, e)})
share = collections.Counter()
busy = 0.0
for a, b in zip(pts, pts[1:]):
    act = [n for s, e, n in ev if s <= a and e >= b]
    if not act:
        continue
    busy += b - a
    for n in act:
        share[n] += (b - a) / len(act)
print(f"window {(hi - lo) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms")
for n, t in share.most_common():
    print(f"{t / 1e6:9.2f} ms {100 * t / busy:5.1f} %  {n}")
