#!/usr/bin/env python3
"""Per-wave time split of the aggregation streamer (experiment build -DTSM_EXP_STAMPS):
loader vmcnt wait / barrier wait / work, for the LAST aggregation pass of a compute."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tea_stereo_matching_amd as tsm
from tea_stereo_matching_amd import _native

H, W, D = 375, 1242, 192
l, r, _ = tsm.synthetic.make_scene(1000, H, W, D + 1)
m = tsm.ADCensus(0)
m.setMatchingStrategy(tsm.ColorModel.RGB, False, False)
m.setMinMaxDisparity(0, D)
for _ in range(2):
    m.compute(l, r)
lib = _native.load()
n = 8192 * 16 * 4
buf = np.zeros(n, dtype=np.uint64)
lib.tsm_exp_agg_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(n * 8))
st = buf.reshape(8192, 16, 4).astype(np.float64)
nb = 2 * W  # last pass of the pipeline: vertical (hf=F on iteration 4 -> vertical second)
used = st[:, :, 0].sum(axis=1) > 0
st = st[used]
print("blocks", st.shape[0])
for w, name in ((0, "summing wave 0"), (11, "summing wave 11"), (12, "loader 0"), (15, "loader 3")):
    a = st[:, w, :]
    print(f"{name:15s} total {a[:,0].mean():9.0f}  vmwait {a[:,1].mean():9.0f}  barrier {a[:,2].mean():9.0f}  work {a[:,3].mean():9.0f}")
