"""Per-pair stage times of one shape / mode (measurement tooling, not the product).

    python3 tools/stage_probe.py --height H --width W --max-disparity D [--hsi] [--omp T]
        [--pairs n] [--concurrency K] [--label name]

Synthetic pairs resident in HBM; pairs/s over two batches of n pairs in groups of K, then
the per-pair stage times with one pipeline alone (groups of one, hipEvents).  The library
is the default one unless TSM_EXPERIMENT_LIB names an experiment build.  Outputs are not
checked (use bench.py / the tests for that)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import tea_stereo_matching_amd as tsm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=375)
    ap.add_argument("--width", type=int, default=1242)
    ap.add_argument("--max-disparity", type=int, default=192)
    ap.add_argument("--hsi", action="store_true")
    ap.add_argument("--omp", type=int, default=0)
    ap.add_argument("--pairs", type=int, default=16)
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--label", default=os.environ.get("TSM_EXPERIMENT_LIB", "default"))
    ap.add_argument("--png", nargs=2, default=None, help="a real pair (tests/golden/demo names), replicated")
    ap.add_argument("--noisy", action="store_true", help="config-B style pairs with +-3 noise on the right view")
    ap.add_argument("--grey", action="store_true", help="grey synthetic scenes (config E)")
    ap.add_argument("--single", type=int, default=0, help="also time N single-frame compute() calls")
    a = ap.parse_args()
    D, n = a.max_disparity, a.pairs
    dev = torch.device("cuda", 0)
    lefts, rights = [], []
    if a.png:
        import numpy as np
        from PIL import Image

        d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "demo")
        ld = lambda f: np.ascontiguousarray(np.array(Image.open(os.path.join(d, f)).convert("RGB"))[:, :, ::-1])  # noqa: E731
        l0, r0 = ld(a.png[0]), ld(a.png[1])
        pairs = [(l0, r0, None)] * n
    elif a.noisy:
        pairs = [tsm.synthetic.config_b_noisy(1000 + i) for i in range(n)]
    else:
        pairs = tsm.synthetic.make_scene_batch([1000 + i for i in range(n)], a.height, a.width, D + 1, threads=16,
                                               grayscale=a.grey)
    H, W = pairs[0][0].shape[:2]
    for l, r, _ in pairs:
        lefts.append(torch.from_numpy(l).to(dev))
        rights.append(torch.from_numpy(r).to(dev))
    outs = torch.empty((n, H, W), dtype=torch.float32, device=dev)
    m = tsm.ADCensus(0)
    m.setMatchingStrategy(tsm.ColorModel.HSI if a.hsi else tsm.ColorModel.RGB, False, False)
    m.setMinMaxDisparity(0, D)
    if a.omp:
        m.setOmpEmulation(a.omp)
    lp = [t.data_ptr() for t in lefts]
    rp = [t.data_ptr() for t in rights]
    op = [outs[i].data_ptr() for i in range(n)]
    m.setConcurrency(a.concurrency)
    m.compute_batch_device_ptr(lp, rp, H, W, W * 3, op, W * 4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2):
        m.compute_batch_device_ptr(lp, rp, H, W, W * 3, op, W * 4)
    torch.cuda.synchronize()
    pps = 2 * n / (time.perf_counter() - t0)
    m.setConcurrency(1)
    single = None
    if a.single:
        m.compute_device_ptr(lp[0], rp[0], H, W, W * 3, op[0], W * 4)
        m.synchronize()
        t1 = time.perf_counter()
        for i in range(a.single):
            m.compute_device_ptr(lp[i % n], rp[i % n], H, W, W * 3, op[i % n], W * 4)
            m.synchronize()
        single = round((time.perf_counter() - t1) / a.single * 1e3, 3)
    m.setProfiling(True)
    m.resetStageTimes()
    k = min(n, 8)
    m.compute_batch_device_ptr(lp[:k], rp[:k], H, W, W * 3, op[:k], W * 4)
    torch.cuda.synchronize()
    st = m.stageTimes()
    m.close()
    print(a.label, f"{W}x{H} D={D}{' HSI' if a.hsi else ''}", round(pps, 2), f"single_ms={single}",
          json.dumps({kk: round(v[0] / max(1, v[1]), 4) for kk, v in st.items()}), flush=True)


if __name__ == "__main__":
    main()
