"""Do the aggregation streamer's blocks land on the XCDs its line order assumes? (measurement
tooling, not the product)

    TSM_EXPERIMENT_LIB=build/exp/agg_xcc/libtsm_adcensus.so python3 tools/xcc_probe.py [--handles N]

The headline batch (config B, 128 pairs, groups of 64 on the two group streams) on N fresh
handles in turn; after each handle's batches, the probe build's record of every block's XCD
(y = 0, pair 0, each group's last fused launch; tools/probes/agg_xcc.patch) gives, per
group, the share of blocks b whose XCD is (b + c) mod 8 for the launch's most common c: 1.0
when the blocks were dealt round-robin from one start, as xcd_remap assumes."""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import tea_stereo_matching_amd as tsm  # noqa: E402
from tea_stereo_matching_amd import _native as Nn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--handles", type=int, default=6)
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--shift-gb", type=float, default=0.0, help="hold this much HBM before the first handle")
    ap.add_argument("--streams", type=int, default=0, help="create this many streams before the first handle")
    a = ap.parse_args()
    H, W, D, n = 375, 1242, 192, 128
    dev = torch.device("cuda", 0)
    pairs = tsm.synthetic.make_scene_batch(range(1000, 1000 + n), H, W, D + 1, threads=16)
    lefts = [torch.from_numpy(l).to(dev) for l, _, _ in pairs]
    rights = [torch.from_numpy(r).to(dev) for _, r, _ in pairs]
    outs = torch.empty((n, H, W), dtype=torch.float32, device=dev)
    lp = [t.data_ptr() for t in lefts]
    rp = [t.data_ptr() for t in rights]
    op = [outs[i].data_ptr() for i in range(n)]
    hold = torch.empty(int(a.shift_gb * 2**30), dtype=torch.uint8, device=dev) if a.shift_gb > 0 else None
    extra = [torch.cuda.Stream(dev) for _ in range(a.streams)]
    for x in extra:
        with torch.cuda.stream(x):
            torch.ones(1, device=dev).add_(1)
    torch.cuda.synchronize()
    lib = Nn.load()
    rec = np.zeros((8, 4096), np.uint32)
    probe = hasattr(lib, "tsm_probe_xcc")  # only the agg_xcc probe build records the XCDs
    if probe:
        lib.tsm_probe_xcc(rec.ctypes.data_as(ctypes.c_void_p), 1)
    for h in range(a.handles):
        m = tsm.ADCensus(0)
        m.setMatchingStrategy(tsm.ColorModel.RGB, False, False)
        m.setMinMaxDisparity(0, D)
        m.setConcurrency(a.concurrency)
        m.compute_batch_device_ptr(lp, rp, H, W, W * 3, op, W * 4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.batches):
            m.compute_batch_device_ptr(lp, rp, H, W, W * 3, op, W * 4)
        torch.cuda.synchronize()
        pps = n * a.batches / (time.perf_counter() - t0)
        if probe:
            rc = lib.tsm_probe_xcc(rec.ctypes.data_as(ctypes.c_void_p), 1)
            assert rc == 0, rc
        m.close()
        out = []
        for s in range(8 if probe else 0):
            r = rec[s]
            if not (r[0] & 0x100):
                continue
            G = int(r[0] >> 16)
            x = (r[:G] & 15).astype(np.int64)
            d = (x - np.arange(G)) & 7
            c = np.bincount(d, minlength=8)
            out.append(f"slot {s}: G {G}, aligned {c.max() / G:.2f} (offsets {c.tolist()})")
        print(f"handle {h}: {pps:7.2f} pairs/s; " + "; ".join(out), flush=True)


if __name__ == "__main__":
    main()
