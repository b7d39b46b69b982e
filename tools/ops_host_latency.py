#!/usr/bin/env python3
"""Host-form latency of the f2-f4 operators (numpy in, numpy out) on a config-B-sized
disparity / image: what a drop-in caller of applyColorMap / reprojectToDepth /
reprojectTo3D / remap pays per call, copies included."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import tea_stereo_matching_amd as T  # noqa: E402

H, W = 375, 1242
rng = np.random.default_rng(0)
disp = (rng.random((H, W), dtype=np.float32) * 190).astype(np.float32)
img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
mx = np.tile(np.arange(W, dtype=np.float32) + 0.3, (H, 1))
my = np.tile(np.arange(H, dtype=np.float32)[:, None] + 0.2, (1, W))


def t(name, fn, n=20):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    print(f"{name}: {(time.perf_counter() - t0) / n * 1e3:.3f} ms/call")


t("applyColorMap", lambda: T.applyColorMap(disp))
t("reprojectToDepth", lambda: T.reprojectToDepth(disp, 700.0, 0.12))
t("reprojectTo3D", lambda: T.reprojectTo3D(disp, 700.0, 0.12, 620.0, 187.0))
t("remap", lambda: T.remap(img, mx, my))
