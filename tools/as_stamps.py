#!/usr/bin/env python3
"""Per-wave time split of the v5 aggregation streamer (experiment build -DTSM_EXP_STAMPS),
last FUSED launch of a compute: summing waves [barrier, pass A, pass B, total],
loaders [barrier, land, issue, total] in s_memtime ticks."""
import ctypes, os, sys, time
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
n = 1024 * 16 * 4
buf = np.zeros(n, dtype=np.uint64)
lib.tsm_exp_as_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(n * 8))
st = buf.reshape(1024, 16, 4).astype(np.float64)
used = st[:, :, 3].sum(axis=1) > 0
st = st[used]
print("blocks", st.shape[0])
for w in (0, 3, 7, 8, 11, 15):
    a = st[:, w, :]
    name = f"A wave {w}" if w < 8 else f"B wave {w-8}"
    print(f"{name:12s} barrier {a[:,0].mean():9.0f}  A/land {a[:,1].mean():9.0f}  B/issue {a[:,2].mean():9.0f}  total {a[:,3].mean():9.0f}")
