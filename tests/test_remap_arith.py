"""The f4 remap kernel's arithmetic (k_stereo_ops.hip remap_tap / remap_apply), restated in
numpy and checked against the reference formula on the CPU: cv::remap INTER_LINEAR with
CV_16SC2 + CV_16UC1 maps computes sum_ij t_ij * w_ij + 2^14 >> 15 with Q15 weights
w = (32-fx | fx) x (32-fy | fy) * 32 (oracle/stereo_ops.c, EpipolarRectify.cpp:87-101).
The kernel forms per channel the column sums v = t0 * wy0 + t1 * wy1 in 16-bit lanes
(v_pk_mad_u16), then one 2-term dot product with the horizontal weights scaled by 64 plus
512 << 6 (v_dot2_u32_u16), and takes byte 2.  Border taps carry weight 0."""
import numpy as np


def reference(t, fx, fy):
    t00, t01, t10, t11 = (t[..., k].astype(np.int64) for k in range(4))
    w00 = (32 - fx) * (32 - fy) * 32
    w01 = fx * (32 - fy) * 32
    w10 = (32 - fx) * fy * 32
    w11 = fx * fy * 32
    return (t00 * w00 + t01 * w01 + t10 * w10 + t11 * w11 + (1 << 14)) >> 15


def kernel_form(t, fx, fy, ra=True, rb=True, c0=True, c1=True):
    """remap_apply with the weights remap_tap gives: a row outside the image gets vertical
    weight 0 (ra / rb), a column outside gets horizontal weight 0 (c0 / c1)."""
    u16 = lambda a: a & 0xFFFF  # noqa: E731  (16-bit lanes of v_pk_mad_u16)
    wa = np.where(ra, 32 - fy, 0)
    wb = np.where(rb, fy, 0)
    ws0 = np.where(c0, 32 - fx, 0)
    ws1 = np.where(c1, fx, 0)
    v0 = u16(u16(t[..., 0] * wa) + u16(t[..., 2] * wb))  # slot 0: rows a, b
    v1 = u16(u16(t[..., 1] * wa) + u16(t[..., 3] * wb))  # slot 1
    d = (v0 * (ws0 << 6) + v1 * (ws1 << 6) + (512 << 6)) & 0xFFFFFFFF
    assert np.all(d < (1 << 24)), "the result must sit in byte 2 with byte 3 clear"
    return (d >> 16) & 0xFF


def test_kernel_form_equals_reference_random():
    rng = np.random.default_rng(0)
    n = 1_000_000
    t = rng.integers(0, 256, (n, 4))
    fx = rng.integers(0, 32, n)
    fy = rng.integers(0, 32, n)
    assert np.array_equal(kernel_form(t, fx, fy), reference(t, fx, fy))


def test_kernel_form_equals_reference_extremes():
    # every fraction pair against every tap pattern of 0 / 255 (the rounding edges)
    fx, fy = np.meshgrid(np.arange(32), np.arange(32), indexing="ij")
    fx, fy = fx.ravel(), fy.ravel()
    for pat in range(16):
        t = np.array([255 if (pat >> k) & 1 else 0 for k in range(4)])[None, :].repeat(fx.size, 0)
        assert np.array_equal(kernel_form(t, fx, fy), reference(t, fx, fy))
    for v in (1, 127, 128, 254):
        t = np.full((fx.size, 4), v)
        assert np.array_equal(kernel_form(t, fx, fy), reference(t, fx, fy))


def test_border_taps_weighted_zero_equal_constant_border():
    # BORDER_CONSTANT 0: tap (row, column) is inside iff its row and its column are, and a
    # tap outside contributes as a 0-valued tap
    rng = np.random.default_rng(1)
    n = 200_000
    t = rng.integers(0, 256, (n, 4))
    fx = rng.integers(0, 32, n)
    fy = rng.integers(0, 32, n)
    ra, rb, c0, c1 = (rng.integers(0, 2, n).astype(bool) for _ in range(4))
    inside = np.stack([ra & c0, ra & c1, rb & c0, rb & c1], -1)
    got = kernel_form(t, fx, fy, ra, rb, c0, c1)
    assert np.array_equal(got, reference(np.where(inside, t, 0), fx, fy))
