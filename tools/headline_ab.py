"""Same-process A/B of the headline batch (measurement tooling, not the product).

    python3 tools/headline_ab.py [--reps R] [--batches K]

Config B: 128 synthetic pairs (seeds 1000..1127) resident in HBM, groups of 64 on the two
group streams, as bench.py's timed loop.  Alternates, R times: a long-lived handle (created
once, as bench.py's), a fresh handle each round, and a fresh handle with
setOmpEmulation(20) (bench.py's B_OMP20 leg); each times K synchronous batch calls.
Prints pairs/s per variant and round."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import tea_stereo_matching_amd as tsm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batches", type=int, default=5)
    ap.add_argument("--variants", default="long,fresh,omp20")
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

    def handle(omp=0):
        m = tsm.ADCensus(0)
        m.setMatchingStrategy(tsm.ColorModel.RGB, False, False)
        m.setMinMaxDisparity(0, D)
        m.setOmpEmulation(omp)
        m.setConcurrency(64)
        return m

    def timed(m, k):
        m.compute_batch_device_ptr(lp, rp, H, W, W * 3, op, W * 4)
        torch.cuda.synchronize()
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            m.compute_batch_device_ptr(lp, rp, H, W, W * 3, op, W * 4)
            ts.append(time.perf_counter() - t0)
        return n * k / sum(ts), min(ts) * 1e3, max(ts) * 1e3

    long_m = None  # created at its first use
    for r in range(a.reps):
        for v in a.variants.split(","):
            if v == "long":
                long_m = long_m or handle()
                m = long_m
            else:
                m = handle(20 if v == "omp20" else 0)
            pps, lo, hi = timed(m, a.batches)
            if m is not long_m:
                m.close()
            print(f"round {r} {v:6s} {pps:8.2f} pairs/s  step {lo:.1f}-{hi:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
