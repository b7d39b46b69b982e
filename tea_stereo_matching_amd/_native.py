"""Loader for the gfx950 AD-Census library (libtsm_adcensus.so) and its C ABI.

The library is built in-tree (``make lib`` / ``__graft_entry__.build()``).  There is no
fallback: if the shared object is missing, importing the bindings raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libtsm_adcensus.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "tsm_adcensus.h")
OPS_HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "tsm_stereo_ops.h")

TSM_OK = 0
TSM_ERR_ARGUMENT = -1
TSM_ERR_DISPARITY_RANGE = -2
TSM_ERR_OFFSET = -3
TSM_ERR_IMAGE = -4
TSM_ERR_DEVICE = -5
TSM_ERR_OUT_OF_MEMORY = -6
TSM_ERR_UNSUPPORTED = -7

STAGES = ("prep", "cost", "arms", "aggregate", "scanline", "refine")

_P = ctypes.c_void_p


class TsmParams(ctypes.Structure):
    """tsm_adc_params (mirrors stereo::ADCensusParams, stereo_utils.h:209-244)."""

    _fields_ = [
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
    ]


class TsmDump(ctypes.Structure):
    _fields_ = [(n, _P) for n in (
        "images", "cost_init", "arms", "cost_agg", "cost_scan", "wta", "outlier",
        "voting", "interp", "gray", "edges", "adjusted", "subpix")]


# name -> (restype, argtypes); every symbol include/tsm_adcensus.h declares
SIGNATURES = {
    "tsm_adc_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    "tsm_adc_destroy": (ctypes.c_int, [_P]),
    "tsm_adc_set_disparity_range": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int]),
    "tsm_adc_set_strategy": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "tsm_adc_set_offset": (ctypes.c_int, [_P, ctypes.c_int]),
    "tsm_adc_compute": (ctypes.c_int, [_P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                       _P, ctypes.c_size_t]),
    "tsm_adc_compute_device": (ctypes.c_int, [_P, _P, _P, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_size_t, _P, ctypes.c_size_t, _P]),
    "tsm_adc_compute_batch": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_size_t, _P, ctypes.c_size_t]),
    "tsm_adc_compute_batch_device": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, ctypes.c_int,
                                                    ctypes.c_int, ctypes.c_size_t, _P,
                                                    ctypes.c_size_t]),
    "tsm_adc_synchronize": (ctypes.c_int, [_P]),
    "tsm_adc_get_params": (ctypes.c_int, [_P, ctypes.POINTER(TsmParams)]),
    "tsm_adc_set_params": (ctypes.c_int, [_P, ctypes.POINTER(TsmParams)]),
    "tsm_adc_get_disparity_range": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int),
                                                   ctypes.POINTER(ctypes.c_int)]),
    "tsm_adc_set_concurrency": (ctypes.c_int, [_P, ctypes.c_int]),
    "tsm_adc_set_omp_emulation": (ctypes.c_int, [_P, ctypes.c_int]),
    "tsm_adc_compute_debug": (ctypes.c_int, [_P, _P, _P, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_size_t, _P, ctypes.c_size_t,
                                             ctypes.POINTER(TsmDump)]),
    "tsm_adc_set_profiling": (ctypes.c_int, [_P, ctypes.c_int]),
    "tsm_adc_stage_times": (ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    "tsm_adc_reset_stage_times": (ctypes.c_int, [_P]),
    "tsm_adc_workspace_bytes": (ctypes.c_size_t, [_P, ctypes.c_int, ctypes.c_int]),
    "tsm_adc_convert_hsi": (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                           _P, ctypes.c_size_t]),
    "tsm_adc_last_error": (ctypes.c_char_p, [_P]),
    "tsm_device_count": (ctypes.c_int, []),
    "tsm_version": (ctypes.c_char_p, []),
}

_i, _z, _f = ctypes.c_int, ctypes.c_size_t, ctypes.c_float
# every symbol include/tsm_stereo_ops.h declares
OPS_SIGNATURES = {
    "tsm_jet_colormap": (_i, [_P]),
    "tsm_stream_synchronize": (_i, [_P]),
    "tsm_apply_colormap": (_i, [_P, _i, _i, _z, _P, _i, _f, _f, _P, _z]),
    "tsm_apply_colormap_device": (_i, [_P, _i, _i, _z, _P, _i, _f, _f, _P, _z, _P]),
    "tsm_reproject_to_depth": (_i, [_P, _i, _i, _z, _f, _f, _P, _z]),
    "tsm_reproject_to_depth_device": (_i, [_P, _i, _i, _z, _f, _f, _P, _z, _P]),
    "tsm_reproject_to_3d": (_i, [_P, _i, _i, _z, _f, _f, _f, _f, _P, _z]),
    "tsm_reproject_to_3d_device": (_i, [_P, _i, _i, _z, _f, _f, _f, _f, _P, _z, _P]),
    "tsm_reproject_to_3d_q": (_i, [_P, _i, _i, _z, _P, _P, _z]),
    "tsm_reproject_to_3d_q_device": (_i, [_P, _i, _i, _z, _P, _P, _z, _P]),
    "tsm_write_point_cloud_pcd": (_i, [_P, _z, _P, _z, _i, _i, ctypes.c_char_p]),
    "tsm_write_point_cloud_ply": (_i, [_P, _z, _P, _z, _i, _i, ctypes.c_char_p]),
    "tsm_remap_linear_fixed": (_i, [_P, _i, _i, _z, _i, _P, _z, _P, _z, _i, _i, _P, _z]),
    "tsm_remap_linear_fixed_device": (_i, [_P, _i, _i, _z, _i, _P, _z, _P, _z, _i, _i, _P, _z, _P]),
    "tsm_remap_linear_float": (_i, [_P, _i, _i, _z, _i, _P, _P, _z, _i, _i, _P, _z]),
    "tsm_remap_linear_float_device": (_i, [_P, _i, _i, _z, _i, _P, _P, _z, _i, _i, _P, _z, _P]),
    # group forms: n maps through one launch (pointer arrays of device buffers)
    "tsm_apply_colormap_batch_device": (_i, [_i, _P, _i, _i, _z, _P, _i, _f, _f, _P, _z, _P]),
    "tsm_reproject_to_depth_batch_device": (_i, [_i, _P, _i, _i, _z, _f, _f, _P, _z, _P]),
    "tsm_reproject_to_3d_batch_device": (_i, [_i, _P, _i, _i, _z, _f, _f, _f, _f, _P, _z, _P]),
    "tsm_remap_linear_fixed_batch_device": (_i, [_i, _P, _i, _i, _z, _i, _P, _z, _P, _z, _i, _i, _P, _z, _P]),
}

_lib = None
LOADED_PATH = None  # the library file this process loaded (bench.py records it)


def library_path() -> str:
    """The product library, or -- for same-box A/B timing of a `make exp` build only -- the
    file TSM_EXPERIMENT_LIB names.  Overridden loads print a warning on stderr and are
    recorded in bench.py's line (`library`), so no result silently comes from another build."""
    override = os.environ.get("TSM_EXPERIMENT_LIB")
    if override:
        import sys

        print(f"[tea_stereo_matching_amd] WARNING: TSM_EXPERIMENT_LIB loads {override} instead of "
              f"{LIB_PATH}", file=sys.stderr)
        return override
    return LIB_PATH


def load() -> ctypes.CDLL:
    """Load the HIP library (raises if it has not been built: no CPU fallback)."""
    global _lib, LOADED_PATH
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build the gfx950 library first "
            "(`make lib` or `python -c 'import __graft_entry__ as g; g.build()'`)")
    # One HIP runtime per process: torch ships its own libamdhip64 (same soname).  Loaded
    # first, it is the copy the library's DT_NEEDED binds to; loaded after ours, torch
    # would start a second runtime that sees no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in {**SIGNATURES, **OPS_SIGNATURES}.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    LOADED_PATH = os.path.abspath(path)
    return lib


def device_count() -> int:
    return int(load().tsm_device_count())


def version() -> str:
    return load().tsm_version().decode()
