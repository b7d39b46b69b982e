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
    a = ap.parse_args()
    H, W, D, n = a.height, a.width, a.max_disparity, a.pairs
    dev = torch.device("cuda", 0)
    lefts, rights = [], []
    for l, r, _ in tsm.synthetic.make_scene_batch([1000 + i for i in range(n)], H, W, D + 1, threads=16):
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
    m.setProfiling(True)
    m.resetStageTimes()
    k = min(n, 8)
    m.compute_batch_device_ptr(lp[:k], rp[:k], H, W, W * 3, op[:k], W * 4)
    torch.cuda.synchronize()
    st = m.stageTimes()
    m.close()
    print(a.label, f"{W}x{H} D={D}{' HSI' if a.hsi else ''}", round(pps, 2),
          json.dumps({kk: round(v[0] / max(1, v[1]), 4) for kk, v in st.items()}), flush=True)


if __name__ == "__main__":
    main()
