"""SURVEY §8f f2-f4 on a real MI355X: the gfx950 kernels against the oracle
(oracle/stereo_ops.c), host and device entry points, odd sizes and strides, the edge
values the reference's loops meet (negative / inf / NaN disparities, borders).

Bar: bit-exact, except reprojectTo3D(Q), whose reference product is cv::gemm with an
unstated summation order: relative 1e-6 there (fp32, four terms).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_bgr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tsm():
    import tea_stereo_matching_amd as T

    if T.device_count() == 0:
        pytest.fail("no HIP device visible to a -m gpu test")
    return T


def _disp(rng, H, W, invalid=True):
    d = rng.uniform(0, 192, (H, W)).astype(np.float32)
    d[rng.random((H, W)) < 0.1] = np.float32(rng.choice([0.0, 1.0, 64.0, 191.0]))
    if invalid:
        m = rng.random((H, W))
        d[m < 0.05] = -1.0
        d[(m >= 0.05) & (m < 0.08)] = -2.0
        d[(m >= 0.08) & (m < 0.09)] = np.inf
        d[(m >= 0.09) & (m < 0.095)] = np.nan
        d[(m >= 0.095) & (m < 0.1)] = -0.0
    return d


SIZES = [(1, 1), (3, 5), (37, 61), (375, 1242), (64, 1023)]


@pytest.mark.parametrize("H,W", SIZES)
def test_colormap_bit_exact(tsm, oracle, H, W):
    rng = np.random.default_rng(H * 1000 + W)
    d = _disp(rng, H, W)
    lut = tsm.JETColorMap()
    assert np.array_equal(tsm.applyColorMap(d, lut), oracle.apply_colormap_ex(d))
    assert np.array_equal(tsm.applyColorMap(d, 10.0, 150.0, lut),
                          oracle.apply_colormap_ex(d, min_val=10.0, max_val=150.0))
    # a non-JET table goes through unchanged
    gray = np.repeat(np.arange(256, dtype=np.uint8)[:, None], 3, 1)
    assert np.array_equal(tsm.applyColorMap(d, gray), oracle.apply_colormap_ex(d, gray))


def test_colormap_degenerate_ranges(tsm, oracle):
    for d in (np.full((4, 9), 5.0, np.float32), np.full((4, 9), -1.0, np.float32),
              np.array([[np.inf, -1.0, np.nan]], np.float32)):
        assert np.array_equal(tsm.applyColorMap(d, tsm.JETColorMap()), oracle.apply_colormap_ex(d))


def test_colormap_of_gpu_disparity_renders_reference_png(tsm):
    """f2 end to end against the reference's own output: the GPU matcher (T = 20 race
    emulation) + the GPU colour map reproduce demo-output/0600_adcensus.png exactly."""
    d = os.path.join(GOLDEN, "demo")
    left, right = load_bgr(os.path.join(d, "0600-Left.png")), load_bgr(os.path.join(d, "0600-Right.png"))
    m = tsm.ADCensus(0)
    try:
        m.setMatchingStrategy(tsm.ColorModel.RGB, False, False)
        m.setMinMaxDisparity(0, 192)
        m.setOmpEmulation(20)
        disp = m.compute(left, right)
    finally:
        m.close()
    col = tsm.applyColorMap(disp, tsm.JETColorMap())
    ref = load_bgr(os.path.join(d, "0600_adcensus.png"))
    assert np.array_equal(col, ref), f"{(col != ref).any(-1).sum()} pixels differ"


@pytest.mark.parametrize("H,W", SIZES)
def test_reprojection_bit_exact(tsm, oracle, H, W):
    rng = np.random.default_rng(7 * H + W)
    d = _disp(rng, H, W)
    f, b, cx, cy = 721.5377, 0.5327, 609.5593, 172.854
    assert np.array_equal(tsm.reprojectToDepth(d, f, b), oracle.reproject_to_depth(d, f, b), equal_nan=True)
    assert np.array_equal(tsm.reprojectTo3D(d, f, b, cx, cy), oracle.reproject_to_3d(d, f, b, cx, cy),
                          equal_nan=True)


def test_reprojection_q_within_tolerance(tsm, oracle):
    rng = np.random.default_rng(9)
    d = rng.uniform(1, 192, (375, 1242)).astype(np.float32)
    f, b, cx, cy = 721.5377, 0.5327, 609.5593, 172.854
    Q = np.array([[1, 0, 0, -cx], [0, 1, 0, -cy], [0, 0, 0, f], [0, 0, 1 / b, 0]], np.float64)
    np.testing.assert_allclose(tsm.reprojectTo3D(d, Q), oracle.reproject_to_3d_q(d, Q), rtol=1e-6, atol=1e-6)


class _Hip:
    """Device buffers through the HIP runtime the library itself links (not torch's
    bundled copy: two runtimes in one process do not share a device context)."""

    def __init__(self):
        self.rt = ctypes.CDLL("libamdhip64.so.7")
        self.bufs = []

    def put(self, a: np.ndarray) -> ctypes.c_void_p:
        p = ctypes.c_void_p()
        assert self.rt.hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(a.nbytes, 1))) == 0
        self.bufs.append(p)
        assert self.rt.hipMemcpy(p, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes), 1) == 0
        return p

    def get(self, p, like: np.ndarray) -> np.ndarray:
        out = np.empty_like(like)
        assert self.rt.hipDeviceSynchronize() == 0
        assert self.rt.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), p, ctypes.c_size_t(out.nbytes), 2) == 0
        return out

    def free(self):
        for p in self.bufs:
            self.rt.hipFree(p)


def test_device_forms_match_oracle(tsm, oracle):
    from tea_stereo_matching_amd import _native as N

    lib = N.load()
    hip = _Hip()
    try:
        rng = np.random.default_rng(21)
        H, W = 375, 1242
        d = _disp(rng, H, W)
        dd = hip.put(d)
        lut = tsm.JETColorMap()
        col = np.zeros((H, W, 3), np.uint8)
        dc = hip.put(col)
        for rep in range(3):  # repeated launches reuse the per-stream min/max scratch
            assert lib.tsm_apply_colormap_device(dd, H, W, 4 * W, lut.ctypes.data_as(ctypes.c_void_p), 0,
                                                 0.0, 0.0, dc, 3 * W, None) == 0
            assert np.array_equal(hip.get(dc, col), oracle.apply_colormap_ex(d))
        dep = np.zeros((H, W), np.float32)
        dp = hip.put(dep)
        assert lib.tsm_reproject_to_depth_device(dd, H, W, 4 * W, 700.0, 0.5, dp, 4 * W, None) == 0
        assert np.array_equal(hip.get(dp, dep), oracle.reproject_to_depth(d, 700.0, 0.5), equal_nan=True)
        xyz = np.zeros((H, W, 3), np.float32)
        dx = hip.put(xyz)
        assert lib.tsm_reproject_to_3d_device(dd, H, W, 4 * W, 700.0, 0.5, 620.0, 187.0, dx, 12 * W, None) == 0
        assert np.array_equal(hip.get(dx, xyz), oracle.reproject_to_3d(d, 700.0, 0.5, 620.0, 187.0),
                              equal_nan=True)
    finally:
        hip.free()


def _maps(rng, H, W, sh, sw):
    # a smooth warp (rotation + radial term) around the image, reaching past the borders
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    cx, cy = sw / 2, sh / 2
    a = np.float32(0.03)
    r2 = ((xx - cx) ** 2 + (yy - cy) ** 2) / np.float32(max(sw, sh) ** 2)
    k = np.float32(1) + np.float32(0.08) * r2
    mx = (cx + k * (np.cos(a) * (xx - cx) - np.sin(a) * (yy - cy)) * np.float32(sw / W)).astype(np.float32)
    my = (cy + k * (np.sin(a) * (xx - cx) + np.cos(a) * (yy - cy)) * np.float32(sh / H)).astype(np.float32)
    mx += rng.uniform(-0.5, 0.5, mx.shape).astype(np.float32)
    ix = np.rint(mx * np.float32(32)).astype(np.int64)
    iy = np.rint(my * np.float32(32)).astype(np.int64)
    xy = np.stack([ix >> 5, iy >> 5], -1).astype(np.int16)
    fxy = ((iy & 31) * 32 + (ix & 31)).astype(np.uint16)
    return mx, my, xy, fxy


@pytest.mark.parametrize("C", [1, 3, 4])
@pytest.mark.parametrize("H,W", [(1, 1), (17, 23), (375, 1242), (120, 161)])
def test_remap_bit_exact(tsm, oracle, C, H, W):
    rng = np.random.default_rng(C * 100 + H)
    sh, sw = max(H + 3, 2), max(W - 5, 2)
    src = rng.integers(0, 256, (sh, sw, C) if C > 1 else (sh, sw), dtype=np.uint8)
    mx, my, xy, fxy = _maps(rng, H, W, sh, sw)
    assert np.array_equal(tsm.remap(src, xy, fxy), oracle.remap_linear_fixed(src, xy, fxy))
    assert np.array_equal(tsm.remap(src, mx, my), oracle.remap_linear_float(src, mx, my))


@pytest.mark.parametrize("C", [1, 3, 4])
def test_remap_wave_forms(tsm, oracle, C):
    """The fixed-map kernel's two forms in one map: waves whose pixels' taps are all inside
    the image (smooth warp: no clamps or weight selection) and waves with border or scattered
    taps (rows 16..31 over and past the whole image), and a source at a 1-byte offset."""
    import torch

    rng = np.random.default_rng(31 + C)
    H, W, sh, sw = 70, 300, 64, 290
    src = rng.integers(0, 256, (sh, sw, C) if C > 1 else (sh, sw), dtype=np.uint8)
    _, _, xy, fxy = _maps(rng, H, W, sh, sw)
    # rows 16..31 scattered over (and past) the whole image: border waves
    xy[16:32, :, 0] = rng.integers(-10, sw + 10, (16, W))
    xy[16:32, :, 1] = rng.integers(-10, sh + 10, (16, W))
    want = oracle.remap_linear_fixed(src, xy, fxy)
    assert np.array_equal(tsm.remap(src, xy, fxy), want)
    big = torch.empty(src.size + 1, dtype=torch.uint8, device="cuda")
    mis = big[1:].view(src.shape)
    mis.copy_(torch.from_numpy(src).cuda())
    assert mis.data_ptr() % 4 == 1
    got = tsm.remap(mis, torch.from_numpy(xy).cuda(), torch.from_numpy(fxy.view(np.int16)).cuda())
    assert np.array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("C", [1, 3, 4])
@pytest.mark.parametrize("offset", [0, 1, 3])
@pytest.mark.parametrize("sh,sw", [(9, 13), (1, 1), (2, 1), (1, 5)])
def test_remap_last_row_end(tsm, oracle, C, offset, sh, sw):
    """Taps at the very end of the source buffer: the window read of the last row's last
    pixels runs past the image's bytes (those dwords read as 0 and carry weight 0); every
    fraction, columns sw-3 .. sw, rows sh-3 .. sh, the source at a 0/1/3-byte offset."""
    import torch

    rng = np.random.default_rng(77 + C + offset + sh * sw)
    src = rng.integers(1, 256, (sh, sw, C) if C > 1 else (sh, sw), dtype=np.uint8)
    cols = np.arange(sw - 3, sw + 1)
    rws = np.arange(sh - 3, sh + 1)
    fr = np.arange(0, 1024, 37)
    gx, gy, gf = np.meshgrid(cols, rws, fr, indexing="ij")
    xy = np.stack([gx.ravel(), gy.ravel()], -1).astype(np.int16).reshape(1, -1, 2)
    fxy = gf.ravel().astype(np.uint16).reshape(1, -1)
    want = oracle.remap_linear_fixed(src, xy, fxy)
    big = torch.empty(src.size + offset, dtype=torch.uint8, device="cuda")
    dsrc = big[offset:].view(src.shape)
    dsrc.copy_(torch.from_numpy(src).cuda())
    got = tsm.remap(dsrc, torch.from_numpy(xy).cuda(), torch.from_numpy(fxy.view(np.int16)).cuda())
    assert np.array_equal(got.cpu().numpy(), want)
    # the float-map form over the same taps
    mx = (gx.ravel() + (gf.ravel() & 31) / 32.0).astype(np.float32).reshape(1, -1)
    my = (gy.ravel() + (gf.ravel() >> 5) / 32.0).astype(np.float32).reshape(1, -1)
    assert np.array_equal(tsm.remap(src, mx, my), oracle.remap_linear_float(src, mx, my))


def test_remap_wide_step_fallback(tsm, oracle):
    """A source whose row step is past the buffer form's 2^23-byte limit runs the 64-bit
    gather kernels (k_remap_fixed / k_remap_float): same outputs, borders included."""
    from tea_stereo_matching_amd import _native as N

    lib = N.load()
    hip = _Hip()
    try:
        rng = np.random.default_rng(12)
        sh, sw, C = 3, 40, 3
        step = (1 << 23) + 64
        src = rng.integers(0, 256, (sh, sw, C), dtype=np.uint8)
        wide = np.zeros((sh, step), np.uint8)
        wide[:, :sw * C] = src.reshape(sh, -1)
        H, W = 6, 50
        _, _, xy, fxy = _maps(rng, H, W, sh, sw)
        xy[0, :8, 0] = [-2, -1, 0, sw - 2, sw - 1, sw, 5, 7]
        xy[0, :8, 1] = [0, 1, -1, sh - 1, sh - 2, 1, sh, -2]
        mx = rng.uniform(-2, sw + 1, (H, W)).astype(np.float32)
        my = rng.uniform(-2, sh + 1, (H, W)).astype(np.float32)
        ds = hip.put(wide)
        dxy, dfxy, dmx, dmy = hip.put(xy), hip.put(fxy), hip.put(mx), hip.put(my)
        out = np.zeros((H, W, C), np.uint8)
        do = hip.put(out)
        assert lib.tsm_remap_linear_fixed_device(ds, sh, sw, step, C, dxy, 4 * W, dfxy, 2 * W, H, W, do, C * W,
                                                 None) == 0
        assert np.array_equal(hip.get(do, out), oracle.remap_linear_fixed(src, xy, fxy))
        assert lib.tsm_remap_linear_float_device(ds, sh, sw, step, C, dmx, dmy, 4 * W, H, W, do, C * W, None) == 0
        assert np.array_equal(hip.get(do, out), oracle.remap_linear_float(src, mx, my))
    finally:
        hip.free()


def test_remap_float_map_edge_values(tsm, oracle):
    rng = np.random.default_rng(4)
    src = rng.integers(0, 256, (30, 40, 3), dtype=np.uint8)
    mx = rng.uniform(-2, 42, (12, 16)).astype(np.float32)
    my = rng.uniform(-2, 32, (12, 16)).astype(np.float32)
    mx[0, :4] = [np.nan, np.inf, -np.inf, 1e12]
    my[1, :4] = [np.nan, 3e9, -3e9, 0.015625]  # 1/64: a tie at 1/32 resolution (rounds to even)
    mx[2, :3] = [0.015625, 0.046875, 39.99]
    assert np.array_equal(tsm.remap(src, mx, my), oracle.remap_linear_float(src, mx, my))


def test_epipolar_rectify_side_by_side(tsm, oracle):
    rng = np.random.default_rng(8)
    H, W = 96, 128
    left = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    right = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    _, _, xy0, f0 = _maps(rng, H, W, H, W)
    _, _, xy1, f1 = _maps(rng, H, W, H, W)
    m = tsm.EpipolarRectifyMap(map00=xy0, map01=f0, map10=xy1, map11=f1)
    r = tsm.EpipolarRectify(m, (W, H))
    both = r.rectify(np.concatenate([left, right], 1))
    l2, r2 = r.rectify(left, right)
    exp_l, exp_r = oracle.remap_linear_fixed(left, xy0, f0), oracle.remap_linear_fixed(right, xy1, f1)
    assert np.array_equal(l2, exp_l) and np.array_equal(r2, exp_r)
    assert np.array_equal(both, np.concatenate([exp_l, exp_r], 1))


def test_group_forms_equal_single_calls(tsm, oracle):
    """The group forms (one launch per 64 maps) give every map the single call's result:
    70 maps of odd size (a full launch of 64 + 6), each map its own auto colour range."""
    import torch

    rng = np.random.default_rng(77)
    H, W = 37, 61
    ds = [_disp(rng, H, W) for _ in range(70)]
    ds[5][:] = -1.0  # no valid pixel
    dev = [torch.from_numpy(d).cuda() for d in ds]
    lut = tsm.JETColorMap()
    cols = tsm.applyColorMapBatch(dev, lut)
    for d, c in zip(ds, cols):
        assert np.array_equal(c.cpu().numpy(), oracle.apply_colormap_ex(d))
    cols = tsm.applyColorMapBatch(dev, 10.0, 150.0, lut)
    for d, c in zip(ds, cols):
        assert np.array_equal(c.cpu().numpy(), oracle.apply_colormap_ex(d, min_val=10.0, max_val=150.0))
    for d, o in zip(ds, tsm.reprojectToDepthBatch(dev, 721.5, 0.54)):
        assert np.array_equal(o.cpu().numpy(), oracle.reproject_to_depth(d, 721.5, 0.54), equal_nan=True)
    for d, o in zip(ds, tsm.reprojectTo3DBatch(dev, 721.5, 0.54, 30.2, 17.9)):
        assert np.array_equal(o.cpu().numpy(), oracle.reproject_to_3d(d, 721.5, 0.54, 30.2, 17.9), equal_nan=True)
    imgs = [rng.integers(0, 256, (40, 66, 3), dtype=np.uint8) for _ in range(67)]
    yy, xx = np.mgrid[0:H, 0:W]
    ix = (xx * 32 + rng.integers(-40, 40, (H, W))).astype(np.int64)
    iy = (yy * 32 + rng.integers(-40, 40, (H, W))).astype(np.int64)
    xy = np.stack([ix >> 5, iy >> 5], -1).astype(np.int16)
    fxy = ((iy & 31) * 32 + (ix & 31)).astype(np.uint16)
    outs = tsm.remapBatch([torch.from_numpy(i).cuda() for i in imgs], torch.from_numpy(xy).cuda(),
                          torch.from_numpy(fxy.view(np.int16)).cuda())
    for i, o in zip(imgs, outs):
        assert np.array_equal(o.cpu().numpy(), oracle.remap_linear_fixed(i, xy, fxy))


def test_group_forms_reject_bad_tables(tsm):
    from tea_stereo_matching_amd import _native as N

    lib = N.load()
    P = ctypes.c_void_p
    two_null = (P * 2)(None, None)
    assert lib.tsm_apply_colormap_batch_device(2, two_null, 4, 4, 16, None, 0, 0.0, 0.0, two_null, 12, None) == N.TSM_ERR_ARGUMENT
    assert lib.tsm_reproject_to_depth_batch_device(-1, None, 4, 4, 16, 1.0, 1.0, None, 16, None) == N.TSM_ERR_ARGUMENT
    assert lib.tsm_reproject_to_depth_batch_device(0, None, 4, 4, 16, 1.0, 1.0, None, 16, None) == N.TSM_OK


def test_strided_and_offset_maps(tsm, oracle):
    """The kernels' two layouts: packed maps (run as one flat row, vector loads / stores)
    and strided ones (padded rows, maps at 4-B but not 8-B aligned offsets: scalar and
    halfword paths), every result equal to the oracle's."""
    import torch
    from tea_stereo_matching_amd import _native as N

    lib = N.load()
    P = ctypes.c_void_p
    rng = np.random.default_rng(31)
    H, W, n = 29, 53, 5
    ds = [_disp(rng, H, W) for _ in range(n)]
    # maps packed back to back in one buffer from element 1 on: odd maps start 4-B aligned only
    flat = torch.zeros(1 + n * H * W, dtype=torch.float32, device="cuda")
    packed = [flat[1 + i * H * W: 1 + (i + 1) * H * W].view(H, W) for i in range(n)]
    # strided: rows padded to W + 3 floats
    pad = torch.zeros(n, H, W + 3, dtype=torch.float32, device="cuda")
    strided = [pad[i, :, :W] for i in range(n)]
    for i, d in enumerate(ds):
        packed[i].copy_(torch.from_numpy(d))
        strided[i].copy_(torch.from_numpy(d))
    lut = tsm.JETColorMap()
    lp = lut.ctypes.data_as(P)
    arr = lambda ts: (P * len(ts))(*[t.data_ptr() for t in ts])  # noqa: E731
    for src, step in ((packed, 4 * W), (strided, 4 * (W + 3))):
        # outputs: packed from a 2-B offset (colour), padded rows (depth / points)
        cbuf = torch.zeros(2 + n * H * W * 3, dtype=torch.uint8, device="cuda")
        cols = [cbuf[2 + i * H * W * 3: 2 + (i + 1) * H * W * 3] for i in range(n)]
        dep = torch.zeros(n, H, W + 1, dtype=torch.float32, device="cuda")
        xyz = torch.zeros(n, H, 3 * W + 2, dtype=torch.float32, device="cuda")
        assert lib.tsm_apply_colormap_batch_device(n, arr(src), H, W, step, lp, 0, 0.0, 0.0, arr(cols), 3 * W,
                                                   None) == 0
        assert lib.tsm_reproject_to_depth_batch_device(n, arr(src), H, W, step, 700.0, 0.5, arr(list(dep)),
                                                       4 * (W + 1), None) == 0
        assert lib.tsm_reproject_to_3d_batch_device(n, arr(src), H, W, step, 700.0, 0.5, 20.0, 11.0,
                                                    arr(list(xyz)), 4 * (3 * W + 2), None) == 0
        assert lib.tsm_stream_synchronize(None) == 0
        for i, d in enumerate(ds):
            assert np.array_equal(cols[i].cpu().numpy().reshape(H, W, 3), oracle.apply_colormap_ex(d)), (step, i)
            assert np.array_equal(dep[i, :, :W].cpu().numpy(), oracle.reproject_to_depth(d, 700.0, 0.5),
                                  equal_nan=True), (step, i)
            assert np.array_equal(xyz[i, :, :3 * W].cpu().numpy().reshape(H, W, 3),
                                  oracle.reproject_to_3d(d, 700.0, 0.5, 20.0, 11.0), equal_nan=True), (step, i)


def test_group_forms_reject_bad_arguments(tsm):
    """remapBatch refuses what it would otherwise reinterpret (float maps, float sources,
    mismatched map shapes, host maps); applyColorMapBatch refuses a half-given range."""
    import torch

    imgs = [torch.zeros((8, 10, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    xy = torch.zeros((8, 10, 2), dtype=torch.int16, device="cuda")
    fr = torch.zeros((8, 10), dtype=torch.int16, device="cuda")
    assert len(tsm.remapBatch(imgs, xy, fr)) == 2
    bad = [
        (imgs, xy.float(), fr.float()),                       # float maps: remap() only
        ([i.float() for i in imgs], xy, fr),                   # float sources
        (imgs, xy, fr[:, :9].contiguous()),                    # map shapes differ
        (imgs, xy.cpu(), fr.cpu()),                            # host maps
        (imgs, xy[..., 0].contiguous(), fr),                   # map1 not (H, W, 2)
    ]
    for args in bad:
        with pytest.raises(ValueError):
            tsm.remapBatch(*args)
    d = [torch.zeros((4, 5), dtype=torch.float32, device="cuda")]
    with pytest.raises(ValueError):
        tsm.applyColorMapBatch(d, 1.0, None, tsm.JETColorMap())
    with pytest.raises(TypeError):
        tsm.applyColorMapBatch(d, 1.0, tsm.JETColorMap())
