"""GPU box: the f4 group remap (tsm_remap_linear_fixed_batch_device) on 64 config-B-sized
BGR images with the bench's warp, for experiment builds too (TSM_EXPERIMENT_LIB; a label
per argument, outputs checked equal across the runs of one process).  Measurement tooling."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tea_stereo_matching_amd import _native as Nn  # noqa: E402

lib = Nn.load()
H, W, G = 375, 1242, 64
dev = torch.device("cuda:0")
gen = torch.Generator().manual_seed(5)
srcs = [torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, generator=gen).to(dev) for _ in range(G)]
yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
a = np.float32(np.pi / 360)
mx = (W / 2 + np.cos(a) * (xx - W / 2) - np.sin(a) * (yy - H / 2)).astype(np.float32)
my = (H / 2 + np.sin(a) * (xx - W / 2) + np.cos(a) * (yy - H / 2)).astype(np.float32)
ix, iy = np.rint(mx * 32).astype(np.int64), np.rint(my * 32).astype(np.int64)
xy = torch.from_numpy(np.stack([ix >> 5, iy >> 5], -1).astype(np.int16)).to(dev)
fxy = torch.from_numpy(((iy & 31) * 32 + (ix & 31)).astype(np.int16)).to(dev)
arr = lambda ts: (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])  # noqa: E731
sp = arr(srcs)
ref = None
N = H * W
for form in sys.argv[1:] or ["default"]:
    outs = [torch.zeros((H, W, 3), dtype=torch.uint8, device=dev) for _ in range(G)]
    dp = arr(outs)
    fn = lambda: lib.tsm_remap_linear_fixed_batch_device(G, sp, H, W, 3 * W, 3, ctypes.c_void_p(xy.data_ptr()),  # noqa
                                                          4 * W, ctypes.c_void_p(fxy.data_ptr()), 2 * W, H, W, dp,
                                                          3 * W, None)
    assert fn() == 0 and lib.tsm_stream_synchronize(None) == 0
    best = []
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(20):
            fn()
        assert lib.tsm_stream_synchronize(None) == 0
        best.append((time.perf_counter() - t0) / 20 * 1e6)
    us = min(best)
    o = torch.stack(outs).cpu()
    same = "ref" if ref is None else ("same" if torch.equal(o, ref) else "DIFFERENT")
    if ref is None:
        ref = o
    gb = (6 * N + 6 * N * G) / (us * 1e-6) / 1e9
    print(f"form {form}: {us:7.1f} us/call  {gb:7.1f} GB/s (maps once + 6 B/px/image)  frac {gb / 8000:.3f}  {same}",
          flush=True)
