"""Where a fused aggregation step spends its cycles (measurement tooling, not the product).

    TSM_EXPERIMENT_LIB=build/exp/agg_stamps/libtsm_adcensus.so python3 tools/agg_stamps.py [--png L R | --synthetic]

Runs one pair through the pipeline on the stamp build (tools/probes/agg_stamps.patch: every
wave of workgroup 0 of the last fused launch stamps s_memtime at its step start, after its
window sum and before the step barrier) and prints, over the launch's steps: the step
period, each role's window time against its window length, the time from window end to the
barrier (division, ring write / store) and the wait at the barrier.  A diagnostic build:
read its shares, not its length (the stamps' own waits forbid overlaps)."""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import tea_stereo_matching_amd as tsm  # noqa: E402
from tea_stereo_matching_amd import _native as Nn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--png", nargs=2, default=["0600-Left.png", "0600-Right.png"])
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--max-disparity", type=int, default=192)
    a = ap.parse_args()
    if a.synthetic:
        l, r, _ = tsm.synthetic.make_scene(1000, 375, 1242, a.max_disparity + 1)
    else:
        from PIL import Image

        d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "demo")
        ld = lambda f: np.ascontiguousarray(np.array(Image.open(os.path.join(d, f)).convert("RGB"))[:, :, ::-1])  # noqa
        l, r = ld(a.png[0]), ld(a.png[1])
    m = tsm.ADCensus(0)
    m.setMatchingStrategy(tsm.ColorModel.RGB, False, False)
    m.setMinMaxDisparity(0, a.max_disparity)
    m.setConcurrency(1)
    m.compute(l, r)
    m.compute(l, r)
    lib = Nn.load()
    st = np.zeros((16, 2048, 3), np.uint64)
    ln = np.zeros((16, 2048), np.uint32)
    rc = lib.tsm_probe_agg_stamps(st.ctypes.data_as(ctypes.c_void_p), ln.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, rc
    steps = int((st[:, :, 0] > 0).all(axis=0).sum())
    st = st[:, :steps].astype(np.int64)
    ln = ln[:, :steps].astype(np.int64)
    t0, t1, t2 = st[..., 0], st[..., 1], st[..., 2]
    s0 = t0.min(axis=0)
    period = np.diff(s0)
    body = slice(12, steps - 12)  # away from the prologue / epilogue
    print(f"steps {steps}; step period mean {period[body].mean():.0f} median {np.median(period[body]):.0f} (s_memtime ticks)")
    for name, ws in (("A (pass A, ring1 -> ring2)", range(0, 8)), ("B (pass B, ring2 -> HBM)", range(8, 16))):
        w = list(ws)
        win = (t1[w] - t0[w])[:, body]
        post = (t2[w] - t1[w])[:, body]
        wait = (t0[w][:, 1:] - t2[w][:, :-1])[:, body.start:body.stop - 1]
        start = (t0[w] - s0[None, :])[:, body]
        L = ln[w][:, body]
        sel = L > 0
        fit = np.polyfit(L[sel], win[sel], 1) if sel.sum() > 10 else (0, 0)
        print(f"{name}: start lag {start.mean():.0f}, window {win.mean():.0f} (len {L.mean():.1f}; "
              f"{fit[0]:.1f} ticks an element + {fit[1]:.0f}), after window {post.mean():.0f}, barrier wait {wait.mean():.0f}")
    # the step's critical wave: the one whose t2 is last
    last = t2[:, body].argmax(axis=0)
    print("critical wave histogram:", np.bincount(last, minlength=16).tolist())
    crit_len = ln[:, body][last, np.arange(last.size)]
    print(f"critical wave's window len mean {crit_len.mean():.1f}; step max len mean {ln[:, body].max(axis=0).mean():.1f}; "
          f"mean len {ln[:, body][ln[:, body] > 0].mean():.1f}")
    # step length against the step's longest window
    mx = ln[:, body].max(axis=0)
    per = period[body.start:body.stop]
    fit = np.polyfit(mx[:len(per)], per[:len(mx)], 1)
    print(f"step period vs step's longest window: {fit[0]:.1f} ticks an element + {fit[1]:.0f}")
    m.close()


if __name__ == "__main__":
    main()
