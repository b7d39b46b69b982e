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
