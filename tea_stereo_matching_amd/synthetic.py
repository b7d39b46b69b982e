"""Deterministic synthetic stereo pairs for benchmarks and tests.

A scene is a fronto-parallel background at an integer disparity in [8, 24] plus
``n_rects`` rectangles with integer disparities in [8, L-12], drawn near-over-far.
Every layer k has its own texture ``tex_k(x, y)`` (base BGR U[40, 215] + 4x4-cell
block noise +-24 + pixel noise +-6, clamped to u8) addressed in the left view's
coordinates, so the right view is an exact shift of each layer:

  Left(x, y)  = tex_k(x, y)        for the max-disparity layer whose footprint holds (x, y)
  Right(x, y) = tex_k(x + d_k, y)  for the max-disparity layer whose left footprint
                                   holds (x + d_k, y)

which gives exact ground truth and true occlusions.  All randomness is splitmix64 of
(seed, stream, index) so the generator is platform independent.
"""
from __future__ import annotations

import numpy as np

_M64 = (1 << 64) - 1


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_M64)
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(_M64)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(_M64)
    return z ^ (z >> np.uint64(31))


def _rand(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    """uint64 hash of (seed, stream, idx)."""
    with np.errstate(over="ignore"):
        key = (np.uint64(seed) * np.uint64(0x100000001B3) + np.uint64(stream) * np.uint64(0x9E3779B1))
        return _splitmix64(np.asarray(idx, dtype=np.uint64) ^ key)


def _uniform_int(seed, stream, idx, lo, hi) -> np.ndarray:
    """Integers uniform in [lo, hi] (inclusive)."""
    r = _rand(seed, stream, idx)
    return (lo + (r % np.uint64(hi - lo + 1)).astype(np.int64)).astype(np.int64)


def _texture(seed: int, k: int, xs: np.ndarray, ys: np.ndarray) -> np.ndarray:
    """tex_k at integer coordinates (broadcast arrays) -> (..., 3) uint8 BGR."""
    base = _uniform_int(seed, 1000 + k, np.arange(3), 40, 215)
    cx = (xs // 4).astype(np.int64) & 0xFFFFF
    cy = (ys // 4).astype(np.int64) & 0xFFFFF
    cell = (cy << 20) | cx
    px_ = (ys.astype(np.int64) & 0xFFFFF) << 20 | (xs.astype(np.int64) & 0xFFFFF)
    out = np.empty(np.broadcast(xs, ys).shape + (3,), np.int64)
    for c in range(3):
        blk = _uniform_int(seed, 2000 + 16 * k + c, cell, -24, 24)
        pix = _uniform_int(seed, 3000 + 16 * k + c, px_, -6, 6)
        out[..., c] = base[c] + blk + pix
    return np.clip(out, 0, 255).astype(np.uint8)


def make_scene(seed: int, height: int, width: int, num_labels: int, n_rects: int = 12,
               grayscale: bool = False):
    """Return (left BGR, right BGR, gt disparity int32 of the left view)."""
    L = int(num_labels)
    dmax_rect = max(8, L - 12)
    layers = []  # (d, x0, y0, x1, y1) in left coordinates; background covers everything
    dbg = int(_uniform_int(seed, 1, np.arange(1), 8, min(24, max(8, L - 1)))[0])
    layers.append((dbg, 0, 0, width, height))
    r = _uniform_int(seed, 2, np.arange(5 * n_rects), 0, 1 << 30)
    for i in range(n_rects):
        d = 8 + int(r[5 * i] % (dmax_rect - 8 + 1))
        w = 16 + int(r[5 * i + 1] % max(1, width // 3))
        h = 16 + int(r[5 * i + 2] % max(1, height // 3))
        x0 = int(r[5 * i + 3] % max(1, width - w))
        y0 = int(r[5 * i + 4] % max(1, height - h))
        layers.append((d, x0, y0, min(width, x0 + w), min(height, y0 + h)))
    # near-over-far: paint in increasing disparity (stable on the layer index)
    order = sorted(range(len(layers)), key=lambda k: (layers[k][0], k))
    ys, xs = np.mgrid[0:height, 0:width]
    owner_l = np.zeros((height, width), np.int32)
    owner_r = np.zeros((height, width), np.int32)
    for k in order:
        d, x0, y0, x1, y1 = layers[k]
        owner_l[y0:y1, x0:x1] = k
        # right pixel (x, y) sees left-footprint point (x + d, y)
        rx0, rx1 = max(0, x0 - d), max(0, x1 - d)
        if rx1 > rx0:
            owner_r[y0:y1, rx0:rx1] = k
    left = np.empty((height, width, 3), np.uint8)
    right = np.empty((height, width, 3), np.uint8)
    gt = np.empty((height, width), np.int32)
    for k, (d, *_rest) in enumerate(layers):
        ml = owner_l == k
        if ml.any():
            left[ml] = _texture(seed, k, xs[ml], ys[ml])
            gt[ml] = d
        mr = owner_r == k
        if mr.any():
            right[mr] = _texture(seed, k, xs[mr] + d, ys[mr])
    if grayscale:
        g_l = left[..., 1:2].copy()
        g_r = right[..., 1:2].copy()
        left = np.repeat(g_l, 3, axis=2)
        right = np.repeat(g_r, 3, axis=2)
    return left, right, gt


def config_b(seed: int = 1000):
    """1242x375, setMinMaxDisparity(0, 192) -> 193 labels."""
    return make_scene(seed, 375, 1242, 193)


def add_noise(img: np.ndarray, seed: int, amp: int = 3, stream: int = 7000) -> np.ndarray:
    """img + independent integer noise U[-amp, amp] per pixel and channel (splitmix64 of
    (seed, stream, index)), clamped to u8.  Added to one view only, it breaks the exact
    shift of the synthetic pairs, so no aggregated cost at the true disparity is exactly 0
    -- the property of real pairs that decides how many vectors the scanline stores
    (ADCensus.cpp:880-881 leaves a pixel untouched when its predecessor's minimum is 0)."""
    idx = np.arange(img.size, dtype=np.uint64)
    n = _uniform_int(seed, stream, idx, -amp, amp).reshape(img.shape)
    return np.clip(img.astype(np.int64) + n, 0, 255).astype(np.uint8)


def config_b_noisy(seed: int = 1000, amp: int = 3):
    """config B pair `seed` with independent +-amp noise on the right view (bench B_noisy)."""
    left, right, gt = config_b(seed)
    return left, add_noise(right, seed, amp), gt


def config_c(seed: int = 2000):
    """1500x1000, setMinMaxDisparity(0, 256) -> 257 labels."""
    return make_scene(seed, 1000, 1500, 257)


def config_e(seed: int = 3000):
    """2048x1536 grey replicated to BGR, setMinMaxDisparity(0, 320)."""
    return make_scene(seed, 1536, 2048, 321, grayscale=True)


def make_scene_batch(seeds, height: int, width: int, num_labels: int, threads: int = 8, **kw):
    """make_scene(seed, ...) for every seed, generated on a thread pool (numpy releases the
    GIL): [(left, right, gt), ...] in seed order."""
    from concurrent.futures import ThreadPoolExecutor

    seeds = list(seeds)
    with ThreadPoolExecutor(max(1, min(threads, len(seeds)))) as ex:
        return list(ex.map(lambda s: make_scene(s, height, width, num_labels, **kw), seeds))


def config_b_batch(seeds, threads: int = 8):
    """config_b(seed) for every seed (make_scene_batch)."""
    return make_scene_batch(seeds, 375, 1242, 193, threads)
