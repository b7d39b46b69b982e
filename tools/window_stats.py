"""Cross-window statistics of a real pair (analysis tooling, CPU only, not the product).

    python3 tools/window_stats.py [left.png right.png]      (tests/golden/demo names)

Arms by the reference's computeLimit rule (ADCensus.cpp:604-659, RGB defaults: colour
thresholds 20 / 6, maxLength1 34, maxLength2 17; one shorter where the walk meets the image
border), vectorised over pixels.  Prints, per pass direction, the mean 1-D window length and
the step statistics of the aggregation streamer's work assignment (chunks of 8 pixels along
a line, one window a wave; a fused step sums pass A of chunk s and pass B of chunk s - 6):
the mean of a step's longest window against the mean window, i.e. what the per-step barrier
costs when each step pays its longest window."""
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(name):
    path = os.path.join(ROOT, "tests", "golden", "demo", name)
    return np.ascontiguousarray(np.array(Image.open(path).convert("RGB"))[:, :, ::-1]).astype(np.int32)


def color_diff(a, b):
    return np.abs(a - b).max(axis=-1)


def arm(img, dy, dx, t1=20, t2=6, l1=34, l2=17):
    """computeLimit along (dy, dx) for every pixel (numpy restatement of :604-659)."""
    H, W, _ = img.shape
    yy, xx = np.mgrid[0:H, 0:W]
    avail = np.where(dy < 0, yy, np.where(dy > 0, H - 1 - yy, 0)) if dy else np.where(dx < 0, xx, W - 1 - xx)
    d = np.ones((H, W), np.int32)
    go = avail >= 1
    anyv = go.copy()
    prev = img.copy()
    for step in range(1, l1 + 2):
        if not go.any():
            break
        y1 = np.clip(yy + dy * step, 0, H - 1)
        x1 = np.clip(xx + dx * step, 0, W - 1)
        p1 = img[y1, x1]
        cdp = color_diff(img, p1)
        cond = (cdp < t1) & (color_diff(p1, prev) < t1) & ((step <= l2) | (cdp < t2)) & (step < l1) & \
            (step + 1 <= avail)
        prev = np.where(go[..., None], p1, prev)
        d = np.where(go, step + 1, d)
        go = go & cond
    d = np.where(anyv, d - 1, d)
    return d - 1


def stats(lo, hi, axis):
    """window lengths along lines (axis 1: rows, horizontal pass; 0: columns)."""
    win = (lo + hi + 1).astype(np.int32)
    lines = win if axis == 1 else win.T
    n = lines.shape[1]
    cpl = (n + 7) // 8
    pad = np.zeros((lines.shape[0], cpl * 8), np.int32)
    pad[:, :n] = lines
    chunks = pad.reshape(-1, 8)  # every line's chunks in order (one view)
    a = chunks.max(axis=1)
    b = np.concatenate([np.zeros(6, np.int32), a[:-6]])  # pass B lags 6 chunks
    step_max = np.maximum(a, b)
    return {"mean": float(win.mean()), "p90": float(np.percentile(win, 90)), "max": int(win.max()),
            "step_max_mean": float(step_max.mean()), "chunk_max_mean": float(a.mean())}


def main():
    ln, rn = (sys.argv[1], sys.argv[2]) if len(sys.argv) > 2 else ("0600-Left.png", "0600-Right.png")
    for name in (ln, rn):
        img = load(name)
        up, down = arm(img, -1, 0), arm(img, 1, 0)
        left, right = arm(img, 0, -1), arm(img, 0, 1)
        print(name, "horizontal", stats(left, right, 1))
        print(name, "vertical  ", stats(up, down, 0))


if __name__ == "__main__":
    main()
