#!/usr/bin/env python3
"""Per-stream busy time and cross-stream overlap from a rocprofv3 kernel trace (measurement
tooling, not the product).  For every stream: its hardware queue, dispatches, span and busy
time; for every pair of streams whose spans overlap by more than half of the shorter one (a
handle's two group streams), the time both had a kernel running against the time either did.
usage: stream_overlap.py <kernel_trace.csv> [min_dispatches]"""
import collections
import csv
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def total(u):
    return sum(e - s for s, e in u)


def inter(a, b):
    i = j = 0
    t = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            t += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return t


rows = list(csv.DictReader(open(sys.argv[1])))
mind = int(sys.argv[2]) if len(sys.argv) > 2 else 50
by = collections.defaultdict(list)
q = {}
for r in rows:
    sid = int(r["Stream_Id"])
    by[sid].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    q.setdefault(sid, set()).add(int(r["Queue_Id"]))
st = {s: union(v) for s, v in by.items() if len(v) >= mind}
t0 = min(u[0][0] for u in st.values())
print(f"{'stream':>6s} {'queue':>8s} {'disp':>6s} {'start ms':>9s} {'span ms':>8s} {'busy ms':>8s}")
for s in sorted(st):
    u = st[s]
    print(f"{s:6d} {','.join(map(str, sorted(q[s]))):>8s} {len(by[s]):6d} {(u[0][0] - t0) / 1e6:9.1f} "
          f"{(u[-1][1] - u[0][0]) / 1e6:8.1f} {total(u) / 1e6:8.1f}")
ss = sorted(st)
for i, a in enumerate(ss):
    for b in ss[i + 1:]:
        A, B = st[a], st[b]
        lo, hi = max(A[0][0], B[0][0]), min(A[-1][1], B[-1][1])
        shorter = min(A[-1][1] - A[0][0], B[-1][1] - B[0][0])
        if hi - lo < 0.5 * shorter:
            continue
        both = inter(A, B)
        either = total(union([tuple(x) for x in A] + [tuple(x) for x in B]))
        print(f"streams {a},{b} (queues {sorted(q[a])},{sorted(q[b])}): both running {both / 1e6:.1f} ms, "
              f"either {either / 1e6:.1f} ms, overlap {both / max(1, either):.2f}")
