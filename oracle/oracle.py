"""ctypes wrapper over oracle/build/liboracle_adcensus.so.

TEST INFRASTRUCTURE ONLY: the CPU restatement of the reference AD-Census path
(source/ADCensus.cpp) used as the parity checker.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module.  The product package
(tea_stereo_matching_amd) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle_adcensus.so")

RGB, HSI = 0, 1


class OrcParams(ctypes.Structure):
    _fields_ = [
        ("color_model", ctypes.c_int), ("roi_matching", ctypes.c_int),
        ("mask_matching", ctypes.c_int), ("offset", ctypes.c_int),
        ("min_disparity", ctypes.c_int), ("max_disparity", ctypes.c_int),
        ("lambda_ad", ctypes.c_float), ("census_win", ctypes.c_int),
        ("lambda_census", ctypes.c_float), ("lambda_hue", ctypes.c_float),
        ("lambda_saturation", ctypes.c_float), ("lambda_intensity", ctypes.c_float),
        ("color_thresh1", ctypes.c_int), ("color_thresh2", ctypes.c_int),
        ("saturation_thresh1", ctypes.c_int), ("saturation_thresh2", ctypes.c_int),
        ("intensity_thresh1", ctypes.c_int), ("intensity_thresh2", ctypes.c_int),
        ("max_length1", ctypes.c_int), ("max_length2", ctypes.c_int),
        ("iterations", ctypes.c_int), ("color_diff", ctypes.c_int),
        ("pi1", ctypes.c_float), ("pi2", ctypes.c_float),
        ("disp_tolerance", ctypes.c_int), ("voting_thresh", ctypes.c_int),
        ("voting_ratio_thresh", ctypes.c_float), ("max_search_depth", ctypes.c_int),
        ("blur_kernel_size", ctypes.c_int), ("canny_thresh1", ctypes.c_int),
        ("canny_thresh2", ctypes.c_int), ("canny_kernel_size", ctypes.c_int),
        ("num_threads", ctypes.c_int), ("scan_emulate_threads", ctypes.c_int),
    ]


_P = ctypes.c_void_p


class OrcDump(ctypes.Structure):
    _fields_ = [(n, _P) for n in (
        "images", "cost_init", "arms", "cost_agg", "cost_scan", "wta", "outlier",
        "voting", "interp", "gray", "edges", "adjusted", "subpix")]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.orc_compute.restype = ctypes.c_int
        _lib.orc_compute.argtypes = [ctypes.POINTER(OrcParams), _P, _P, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_size_t, _P, ctypes.POINTER(OrcDump)]
        _lib.orc_default_params.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int]
        for name in ("orc_cv_equalize_hist", "orc_cv_blur3"):
            getattr(_lib, name).argtypes = [_P, _P, ctypes.c_int, ctypes.c_int]
        _lib.orc_cv_canny.argtypes = [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double]
        _lib.orc_cv_median3f.argtypes = [_P, _P, ctypes.c_int, ctypes.c_int]
        _lib.orc_apply_colormap.argtypes = [_P, ctypes.c_int, ctypes.c_int, _P]
        _lib.orc_check_disparity_range.argtypes = [ctypes.c_int, ctypes.c_int]
        _i, _z, _f = ctypes.c_int, ctypes.c_size_t, ctypes.c_float
        _lib.orc_apply_colormap_ex.argtypes = [_P, _i, _i, _z, _P, _i, _f, _f, _P, _z]
        _lib.orc_reproject_depth.argtypes = [_P, _i, _i, _z, _f, _f, _P, _z]
        _lib.orc_reproject_3d.argtypes = [_P, _i, _i, _z, _f, _f, _f, _f, _P, _z]
        _lib.orc_reproject_3d_q.argtypes = [_P, _i, _i, _z, _P, _P, _z]
        _lib.orc_remap_linear_fixed.argtypes = [_P, _i, _i, _z, _i, _P, _z, _P, _z, _i, _i, _P, _z]
        _lib.orc_bgr2hsi.argtypes = [_P, _P, _i, _i, _i]
        _lib.orc_remap_linear_float.argtypes = [_P, _i, _i, _z, _i, _P, _P, _z, _i, _i, _P, _z]
    return _lib


def default_params(color_model: int = RGB, min_d: int = 0, max_d: int = 64, **kw) -> OrcParams:
    p = OrcParams()
    lib().orc_default_params(ctypes.byref(p), color_model)
    p.min_disparity, p.max_disparity = min_d, max_d
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(_P)


def compute(left: np.ndarray, right: np.ndarray, params: OrcParams, dump_stages=()):
    """Run the oracle.  left/right: (H, W, 3) uint8 BGR.  Returns (disparity, dumps)."""
    left = np.ascontiguousarray(left, dtype=np.uint8)
    right = np.ascontiguousarray(right, dtype=np.uint8)
    H, W = left.shape[:2]
    maxd = W // 2 if (params.roi_matching or params.mask_matching) else params.max_disparity
    L = maxd - params.min_disparity + 1
    shapes = {
        "images": ((2, H, W, 3), np.uint8), "cost_init": ((2, L, H, W), np.float32),
        "arms": ((2, 4, H, W), np.int32), "cost_agg": ((2, L, H, W), np.float32),
        "cost_scan": ((2, L, H, W), np.float32), "wta": ((2, H, W), np.int32),
        "outlier": ((H, W), np.int32), "voting": ((H, W), np.int32),
        "interp": ((H, W), np.int32), "gray": ((H, W), np.uint8),
        "edges": ((H, W), np.uint8), "adjusted": ((H, W), np.int32),
        "subpix": ((H, W), np.float32),
    }
    dumps = {k: np.zeros(*shapes[k]) for k in dump_stages}
    d = OrcDump(**{k: _ptr(v) for k, v in dumps.items()})
    out = np.zeros((H, W), np.float32)
    rc = lib().orc_compute(ctypes.byref(params), _ptr(left), _ptr(right), H, W, W * 3, _ptr(out),
                           ctypes.byref(d))
    if rc != 0:
        raise RuntimeError(f"orc_compute failed: {rc}")
    return out, dumps


def bgr2hsi(img: np.ndarray, filter: int = 0) -> np.ndarray:
    """bgr2hsi, ADCensus.cpp:1429-1473 ((H, W, 3) BGR -> H S I bytes)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.zeros_like(img)
    lib().orc_bgr2hsi(_ptr(img), _ptr(out), img.shape[0], img.shape[1], int(filter))
    return out


def apply_colormap(disp: np.ndarray) -> np.ndarray:
    disp = np.ascontiguousarray(disp, dtype=np.float32)
    H, W = disp.shape
    out = np.zeros((H, W, 3), np.uint8)
    lib().orc_apply_colormap(_ptr(disp), H, W, _ptr(out))
    return out


def jet_lut() -> np.ndarray:
    lut = np.zeros((256, 3), np.uint8)
    lib().orc_jet_colormap(_ptr(lut))
    return lut


def canny(src: np.ndarray, low=30.0, high=90.0) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    out = np.zeros_like(src)
    lib().orc_cv_canny(_ptr(src), _ptr(out), src.shape[0], src.shape[1], low, high)
    return out


def blur3(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    out = np.zeros_like(src)
    lib().orc_cv_blur3(_ptr(src), _ptr(out), src.shape[0], src.shape[1])
    return out


def equalize_hist(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    out = np.zeros_like(src)
    lib().orc_cv_equalize_hist(_ptr(src), _ptr(out), src.shape[0], src.shape[1])
    return out


def median3f(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.float32)
    out = np.zeros_like(src)
    lib().orc_cv_median3f(_ptr(src), _ptr(out), src.shape[0], src.shape[1])
    return out


# ---- SURVEY §8f f2-f4 (oracle/stereo_ops.c) ---------------------------------------

def apply_colormap_ex(disp: np.ndarray, lut: np.ndarray | None = None, min_val=None, max_val=None) -> np.ndarray:
    """applyColorMap, stereo.cpp:94-118 (auto range) / :120-134 (min_val, max_val given)."""
    disp = np.ascontiguousarray(disp, dtype=np.float32)
    H, W = disp.shape
    lut = jet_lut() if lut is None else np.ascontiguousarray(lut, dtype=np.uint8)
    out = np.zeros((H, W, 3), np.uint8)
    rng = min_val is not None
    lib().orc_apply_colormap_ex(_ptr(disp), H, W, W, _ptr(lut), int(rng),
                                float(min_val) if rng else 0.0, float(max_val) if rng else 0.0,
                                _ptr(out), W * 3)
    return out


def reproject_to_depth(disp: np.ndarray, f: float, b: float) -> np.ndarray:
    """reprojectToDepth, stereo.cpp:136-148."""
    disp = np.ascontiguousarray(disp, dtype=np.float32)
    H, W = disp.shape
    out = np.zeros((H, W), np.float32)
    lib().orc_reproject_depth(_ptr(disp), H, W, W, f, b, _ptr(out), W)
    return out


def reproject_to_3d(disp: np.ndarray, f: float, b: float, cx: float, cy: float) -> np.ndarray:
    """reprojectTo3D(disparity, f, b, cx, cy), stereo.cpp:150-169."""
    disp = np.ascontiguousarray(disp, dtype=np.float32)
    H, W = disp.shape
    out = np.zeros((H, W, 3), np.float32)
    lib().orc_reproject_3d(_ptr(disp), H, W, W, f, b, cx, cy, _ptr(out), 3 * W)
    return out


def reproject_to_3d_q(disp: np.ndarray, Q: np.ndarray) -> np.ndarray:
    """reprojectTo3D(disparity, Q), stereo.cpp:171-202 (product summed in index order)."""
    disp = np.ascontiguousarray(disp, dtype=np.float32)
    Q = np.ascontiguousarray(Q, dtype=np.float64).reshape(16)
    H, W = disp.shape
    out = np.zeros((H, W, 3), np.float32)
    lib().orc_reproject_3d_q(_ptr(disp), H, W, W, _ptr(Q), _ptr(out), 3 * W)
    return out


def remap_linear_fixed(src: np.ndarray, xy: np.ndarray, fxy: np.ndarray) -> np.ndarray:
    """cv::remap INTER_LINEAR with CV_16SC2 + CV_16UC1 maps (EpipolarRectify.cpp:99-100)."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    C = 1 if src.ndim == 2 else src.shape[2]
    xy = np.ascontiguousarray(xy, dtype=np.int16)
    fxy = np.ascontiguousarray(fxy, dtype=np.uint16)
    H, W = fxy.shape
    out = np.zeros((H, W, C) if C > 1 else (H, W), np.uint8)
    lib().orc_remap_linear_fixed(_ptr(src), src.shape[0], src.shape[1], src.shape[1] * C, C,
                                 _ptr(xy), 2 * W, _ptr(fxy), W, H, W, _ptr(out), W * C)
    return out


def remap_linear_float(src: np.ndarray, mapx: np.ndarray, mapy: np.ndarray) -> np.ndarray:
    """cv::remap INTER_LINEAR with two CV_32FC1 maps."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    C = 1 if src.ndim == 2 else src.shape[2]
    mapx = np.ascontiguousarray(mapx, dtype=np.float32)
    mapy = np.ascontiguousarray(mapy, dtype=np.float32)
    H, W = mapx.shape
    out = np.zeros((H, W, C) if C > 1 else (H, W), np.uint8)
    lib().orc_remap_linear_float(_ptr(src), src.shape[0], src.shape[1], src.shape[1] * C, C,
                                 _ptr(mapx), _ptr(mapy), W, H, W, _ptr(out), W * C)
    return out


def _to_chars_f32(v: np.float32) -> str:
    """std::to_chars(float) (stereo.cpp:234-238): the shortest round-trip digits, printed
    as %f or %e, whichever is shorter (%f on a tie); exponent with at least two digits."""
    v = np.float32(v)
    if np.isnan(v):
        return "-nan" if np.signbit(v) else "nan"
    if np.isinf(v):
        return "-inf" if v < 0 else "inf"
    fx = np.format_float_positional(v, unique=True, trim="-")
    sc = np.format_float_scientific(v, unique=True, trim="-", exp_digits=2)
    return fx if len(fx) <= len(sc) else sc


def point_cloud_text(bgr: np.ndarray, xyz: np.ndarray, kind: str) -> bytes:
    """writePointCloudToPCD / writePointCloudToPLY (stereo.cpp:204-356): points with any
    +inf coordinate are skipped; PCD packs rgb as r<<16 | g<<8 | b | 1<<24."""
    pts = xyz.reshape(-1, 3)
    col = bgr.reshape(-1, 3)
    keep = ~(np.isposinf(pts).any(axis=1))
    pts, col = pts[keep], col[keep]
    n = len(pts)
    if kind == "pcd":
        head = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgb\n"
                "SIZE 4 4 4 4\nTYPE F F F U\nCOUNT 1 1 1 1\n"
                f"WIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\nDATA ascii\n")
        lines = [f"{_to_chars_f32(p[0])} {_to_chars_f32(p[1])} {_to_chars_f32(p[2])} "
                 f"{(int(c[2]) << 16) | (int(c[1]) << 8) | int(c[0]) | (1 << 24)}\n" for p, c in zip(pts, col)]
    else:
        head = ("ply\nformat ascii 1.0\n" f"element vertex {n}\n"
                "property float x\nproperty float y\nproperty float z\n"
                "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")
        lines = [f"{_to_chars_f32(p[0])} {_to_chars_f32(p[1])} {_to_chars_f32(p[2])} "
                 f"{int(c[2])} {int(c[1])} {int(c[0])}\n" for p, c in zip(pts, col)]
    return (head + "".join(lines)).encode()
