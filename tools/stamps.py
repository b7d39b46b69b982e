#!/usr/bin/env python3
"""Timeline of the cost-walk kernel from an experiment build (-DTSM_EXP_STAMPS):
per-wave phase durations (prologue, warm-up, walk) and CU occupancy over time."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tea_stereo_matching_amd as tsm
from tea_stereo_matching_amd import _native

H, W, D = 375, 1242, 192
l, r, _ = tsm.synthetic.make_scene(1000, H, W, D + 1)
m = tsm.ADCensus(0)
m.setMatchingStrategy(tsm.ColorModel.RGB, False, False)
m.setMinMaxDisparity(0, D)
for _ in range(3):
    m.compute(l, r)
lib = _native.load()
n = 65536 * 8
buf = np.zeros(n, dtype=np.uint64)
rc = lib.tsm_exp_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(n * 8)) if hasattr(lib, "tsm_exp_stamps") else -1
st = buf.reshape(-1, 8)
seg = int(os.environ.get("TSM_COST_SEG", "32"))
nseg = (W + seg - 1) // seg
nw = 2 * H * nseg
st = st[:nw]
t0 = st[:, 0].min()
s = (st[:, :4].astype(np.int64) - int(t0))
print("rc", rc, "waves", nw, "kernel span (memtime ticks)", s[:, 3].max())
pro = s[:, 1] - s[:, 0]
warm = s[:, 2] - s[:, 1]
walk = s[:, 3] - s[:, 2]
for name, a in (("prologue", pro), ("warm-up", warm), ("walk", walk), ("start", s[:, 0]), ("end", s[:, 3])):
    print(f"{name:9s} mean {a.mean():10.0f} p10 {np.percentile(a,10):10.0f} p50 {np.median(a):10.0f} p90 {np.percentile(a,90):10.0f} max {a.max():10.0f}")
span = s[:, 3].max()
busy = (s[:, 3] - s[:, 0]).sum()
print("sum of wave lifetimes / span =", busy / span, "(mean resident waves chip-wide)")
# resident waves over time
edges = np.linspace(0, span, 21)
res = [((s[:, 0] <= e) & (s[:, 3] > e)).sum() for e in edges]
print("resident waves at 5% steps:", res)

# --- breakdown of the walk time ---
ids = st[:, 5]
xcc = (ids >> np.uint64(32)).astype(np.int64) & 0xF
hw = (ids & np.uint64(0xFFFFFFFF)).astype(np.int64)
# gfx9 HW_ID: wave_id[3:0], simd_id[5:4], pipe_id[7:6], cu_id[11:8], sh_id[12], se_id[15:13]
simd = (hw >> 4) & 3
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
key = xcc * 100000 + se * 10000 + sh * 1000 + cu * 10 + simd
segi = np.arange(nw) % nseg
view = (np.arange(nw) // nseg) // H
steps_per = np.minimum(seg, W - segi * seg)
per_step = walk / steps_per
print("walk cycles/step by segment index:", [round(float(per_step[segi == k].mean())) for k in range(nseg)])
print("walk cycles/step by view:", [round(float(per_step[view == k].mean())) for k in range(2)])
print("walk cycles/step by xcc:", [round(float(per_step[xcc == k].mean())) for k in range(8)])
uk, cnt = np.unique(key, return_counts=True)
cmap = dict(zip(uk, cnt))
wps = np.array([cmap[k] for k in key])
for c in sorted(set(wps)):
    print(f"waves on this SIMD over the launch = {c}: {np.sum(wps == c)} waves, cycles/step {per_step[wps == c].mean():.0f}")
print("distinct SIMDs used:", len(uk))

# --- per-XCD timeline (s_memtime is per XCD) ---
for x in range(8):
    sel = (xcc == x) & (np.arange(nw) > 0)
    if not sel.any():
        continue
    a = st[sel, :4].astype(np.int64)
    t0x = a[:, 0].min()
    a = a - t0x
    span_x = a[:, 3].max()
    life = (a[:, 3] - a[:, 0]).sum()
    nsimd = len(np.unique(key[sel]))
    edges = np.linspace(0, span_x, 11)
    resid = [int(((a[:, 0] <= e) & (a[:, 3] > e)).sum()) for e in edges[:-1]]
    if x < 2:
        print(f"xcc {x}: span {span_x} cycles, waves {sel.sum()}, SIMDs {nsimd}, mean resident/SIMD {life / span_x / nsimd:.2f}, resident over time {resid}")
