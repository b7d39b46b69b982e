#!/usr/bin/env python3
"""HBM calibration on the GPU box: write-only (fill), read-only (sum) and copy rates
over a buffer the size of one pair's cost volume (both views, config B)."""
import torch

n = 2 * 193 * 1242 * 375  # floats
x = torch.empty(n, dtype=torch.float32, device="cuda")
y = torch.empty_like(x)
x.fill_(1.0)
torch.cuda.synchronize()


def t(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3


b = n * 4
tw = t(lambda: x.fill_(2.0))
tr = t(lambda: x.sum())
tc = t(lambda: y.copy_(x))
print(f"bytes {b/1e6:.1f} MB  write {b/tw/1e9:.0f} GB/s  read {b/tr/1e9:.0f} GB/s  copy(r+w) {2*b/tc/1e9:.0f} GB/s")
