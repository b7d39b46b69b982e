#!/usr/bin/env python3
"""One single-frame call's GPU timeline from a rocprofv3 kernel trace (+ memory-copy trace):
the ops of the last frame (the last `n` kernels before the end of the run, or the kernels
between the last two k_pack_bgr launches), each with start offset, duration and the gap
before it, and totals: busy time, gap time.
usage: frame_timeline.py <kernel_trace.csv> [memory_copy_trace.csv] [--frame K]"""
import csv
import sys


def short(n):
    n = n.split("(")[0]
    for p in ("void ", "tsm::"):
        n = n.replace(p, "")
    return n[:60]


args = [a for a in sys.argv[1:] if not a.startswith("--")]
frame = 2
for a in sys.argv[1:]:
    if a.startswith("--frame="):
        frame = int(a.split("=")[1])
ops = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
       for r in csv.DictReader(open(args[0]))]
if len(args) > 1:
    for r in csv.DictReader(open(args[1])):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    "copy " + r.get("Direction", r.get("Operation", "?"))))
ops.sort()
starts = [i for i, o in enumerate(ops) if o[2].startswith("k_pack_bgr")]
if len(starts) < frame + 1:
    sys.exit("not enough frames in the trace")
a, b = starts[-frame - 1], starts[-frame]
# the frame: from its H2D copies (just before the pack) to the op before the next frame's copies
i0 = a
while i0 > 0 and ops[i0 - 1][2].startswith("copy") and ops[a][0] - ops[i0 - 1][1] < 200_000:
    i0 -= 1
i1 = b
while i1 > a and ops[i1 - 1][2].startswith("copy") and ops[b][0] - ops[i1 - 1][1] < 200_000:
    i1 -= 1
fr = ops[i0:i1]
t0 = fr[0][0]
busy = gap = 0
prev = t0
print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>7}  op")
for s, e, n in fr:
    g = max(0, s - prev)
    gap += g
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {g / 1e3:7.1f}  {n}")
    prev = max(prev, e)
print(f"frame {((prev - t0) / 1e3):.1f} us: busy {busy / 1e3:.1f} us, gaps {gap / 1e3:.1f} us over {len(fr)} ops")
