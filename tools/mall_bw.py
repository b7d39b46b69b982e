#!/usr/bin/env python3
"""Infinity-cache check: in-place read+write rate over working sets of several sizes."""
import torch

for mb in (32, 64, 119, 180, 240, 360, 730):
    n = mb * 1024 * 1024 // 4
    x = torch.ones(n, dtype=torch.float32, device="cuda")
    for _ in range(3):
        x.mul_(1.0000001)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    s.record()
    for _ in range(reps):
        x.mul_(1.0000001)
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / reps / 1e3
    print(f"{mb:4d} MB in-place r+w: {2 * n * 4 / t / 1e9:8.0f} GB/s  ({t*1e6:.0f} us)")
