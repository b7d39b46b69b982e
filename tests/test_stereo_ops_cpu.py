"""SURVEY §8f f2-f4 on the CPU: the oracle restatements against known answers, and the
library's host-only point-cloud writers against the oracle's text restatement.

No kernel runs here (no GPU in the CPU suite); the GPU kernels are checked against the
same oracle in test_gpu_stereo_ops.py.
"""
import numpy as np
import pytest

from tea_stereo_matching_amd import _native as N
import tea_stereo_matching_amd as tsm


# ---- f2 ------------------------------------------------------------------------------

def test_jet_table_matches_reference_loops(oracle):
    # stereo.cpp:75-92: ramps of 4 per index; spot values from the reference's loops
    lut = oracle.jet_lut()
    assert tuple(lut[0]) == (128, 0, 0) and tuple(lut[31]) == (252, 0, 0)
    assert tuple(lut[32]) == (255, 0, 0) and tuple(lut[33]) == (255, 4, 0)
    assert tuple(lut[96]) == (254, 255, 2) and tuple(lut[159]) == (1, 255, 254)
    assert tuple(lut[160]) == (0, 252, 255) and tuple(lut[255]) == (0, 0, 128)


def test_library_jet_table_equals_oracle(oracle):
    assert np.array_equal(tsm.JETColorMap()[0], oracle.jet_lut())


def test_colormap_known_answers(oracle):
    lut = oracle.jet_lut()
    d = np.array([[0.0, 1.0, 2.0, 3.0], [-1.0, -2.0, np.inf, 1.5]], np.float32)
    out = oracle.apply_colormap_ex(d)
    # range [0, 3]: index = (unsigned char)((v - 0) / 3 * 255)
    for (y, x), idx in {(0, 0): 0, (0, 1): 85, (0, 2): 170, (0, 3): 255, (1, 3): 127}.items():
        assert tuple(out[y, x]) == tuple(lut[idx])
    assert not out[1, 0].any() and not out[1, 1].any()  # invalid -> black
    assert tuple(out[1, 2]) == tuple(lut[0])  # +inf: undefined cast, x86 -> index 0
    # explicit range: outside -> black
    out2 = oracle.apply_colormap_ex(d, min_val=1.0, max_val=2.0)
    assert not out2[0, 0].any() and not out2[0, 3].any()
    assert tuple(out2[0, 1]) == tuple(lut[0]) and tuple(out2[0, 2]) == tuple(lut[255])
    assert tuple(out2[1, 3]) == tuple(lut[127])


def test_colormap_constant_map_is_index_zero(oracle):
    # max == min: 0/0 -> NaN index -> x86 0 (the reference's MSVC x64 behaviour)
    d = np.full((3, 5), 7.0, np.float32)
    assert (oracle.apply_colormap_ex(d) == oracle.jet_lut()[0]).all()


# ---- f3 ------------------------------------------------------------------------------

def test_reprojection_known_answers(oracle):
    d = np.array([[2.0, -1.0, np.inf], [4.0, 0.5, 8.0]], np.float32)
    f, b, cx, cy = np.float32(700.0), np.float32(0.12), np.float32(1.0), np.float32(0.5)
    dep = oracle.reproject_to_depth(d, f, b)
    fb = np.float32(f * b)
    assert dep[0, 0] == np.float32(fb / np.float32(2.0)) and dep[0, 1] == 0 and dep[0, 2] == 0
    xyz = oracle.reproject_to_3d(d, f, b, cx, cy)
    Z = np.float32(fb / np.float32(4.0))
    Zf = np.float32(Z / f)
    assert tuple(xyz[1, 0]) == (np.float32((np.float32(0) - cx) * Zf), np.float32((np.float32(1) - cy) * Zf), Z)
    assert not xyz[0, 1].any() and not xyz[0, 2].any()


def test_reprojection_q_matches_explicit_form(oracle):
    # the standard stereoRectify Q: [1 0 0 -cx; 0 1 0 -cy; 0 0 0 f; 0 0 -1/Tx 0] gives
    # X = (u - cx) Z / f, Y = (v - cy) Z / f, Z = f Tx / d  (Tx = -b)
    f, b, cx, cy = 700.0, 0.12, 310.5, 180.25
    Q = np.array([[1, 0, 0, -cx], [0, 1, 0, -cy], [0, 0, 0, f], [0, 0, 1 / b, 0]], np.float64)
    rng = np.random.default_rng(3)
    d = rng.uniform(1, 190, (20, 30)).astype(np.float32)
    a = oracle.reproject_to_3d_q(d, Q)
    e = oracle.reproject_to_3d(d, f, b, cx, cy)
    np.testing.assert_allclose(a, e, rtol=2e-5, atol=1e-5)


# ---- f4 ------------------------------------------------------------------------------

def _grid(H, W):
    xy = np.zeros((H, W, 2), np.int16)
    xy[..., 0] = np.arange(W)[None]
    xy[..., 1] = np.arange(H)[:, None]
    return xy


def test_remap_identity_and_shift(oracle):
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (9, 13, 3), dtype=np.uint8)
    xy = _grid(9, 13)
    z = np.zeros((9, 13), np.uint16)
    assert np.array_equal(oracle.remap_linear_fixed(img, xy, z), img)
    xy2 = xy.copy()
    xy2[..., 0] += 2  # sample x + 2: the last two columns read the border (0)
    out = oracle.remap_linear_fixed(img, xy2, z)
    assert np.array_equal(out[:, :11], img[:, 2:]) and not out[:, 11:].any()


def test_remap_half_pixel_rounds_half_up(oracle):
    img = np.array([[[10], [13]], [[20], [30]]], np.uint8)[..., 0]  # 2x2 grey
    xy = np.zeros((1, 1, 2), np.int16)
    half_x = np.full((1, 1), 16, np.uint16)  # fx = 16 / 32
    assert oracle.remap_linear_fixed(img, xy, half_x)[0, 0] == 12  # (10 + 13 + 1) >> 1
    both = np.full((1, 1), 16 * 32 + 16, np.uint16)
    assert oracle.remap_linear_fixed(img, xy, both)[0, 0] == (10 + 13 + 20 + 30 + 2) // 4


def test_remap_float_maps_equal_fixed_maps(oracle):
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, (40, 50, 3), dtype=np.uint8)
    mx = rng.uniform(-3, 53, (30, 35)).astype(np.float32)
    my = rng.uniform(-3, 43, (30, 35)).astype(np.float32)
    ix = np.rint(mx * np.float32(32)).astype(np.int64)
    iy = np.rint(my * np.float32(32)).astype(np.int64)
    xy = np.stack([ix >> 5, iy >> 5], -1).astype(np.int16)
    f = ((iy & 31) * 32 + (ix & 31)).astype(np.uint16)
    assert np.array_equal(oracle.remap_linear_float(img, mx, my), oracle.remap_linear_fixed(img, xy, f))


# ---- f3 writers: host code of the library ----------------------------------------------

def _cloud(rng, H=7, W=9):
    xyz = rng.normal(0, 50, (H, W, 3)).astype(np.float32)
    xyz[0, 0, 2] = np.inf
    xyz[1, 2, 0] = np.inf
    xyz[2, 3, 1] = -np.inf  # only +inf is skipped (stereo.cpp:268-270)
    xyz[3, 3] = (1e20, 1.5e-7, 100.0)
    xyz[4, 4] = (0.1, -0.0, 123456.7)
    bgr = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    return bgr, xyz


@pytest.mark.parametrize("kind", ["pcd", "ply"])
def test_point_cloud_writer_bytes(oracle, tmp_path, kind):
    rng = np.random.default_rng(11)
    bgr, xyz = _cloud(rng)
    path = str(tmp_path / f"cloud.{kind}")
    (tsm.writePointCloudToPCD if kind == "pcd" else tsm.writePointCloudToPLY)(bgr, xyz, path)
    got = open(path, "rb").read()
    assert got == oracle.point_cloud_text(bgr, xyz, kind)
    n = 7 * 9 - 2
    assert (b"POINTS %d\n" % n in got) if kind == "pcd" else (b"element vertex %d\n" % n in got)


def test_point_cloud_writer_empty_input_is_a_no_op(tmp_path):
    path = tmp_path / "none.pcd"
    tsm.writePointCloudToPCD(np.zeros((0, 0, 3), np.uint8), np.zeros((0, 0, 3), np.float32), str(path))
    assert not path.exists()
    assert N.load().tsm_write_point_cloud_ply(None, 0, None, 0, 1, 1, b"x") == N.TSM_ERR_ARGUMENT


def test_rectify_requires_maps():
    r = tsm.EpipolarRectify()
    assert r.rectify(np.zeros((4, 8, 3), np.uint8)) is None  # logs + returns (EpipolarRectify.cpp:48-52)
    with pytest.raises(RuntimeError, match="stereo params is empty"):
        r.loadEpipolarRectifyMap(tsm.EpipolarRectifyMap(), (4, 4))
