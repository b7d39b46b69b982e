"""The C-ABI library loads and exports every symbol include/tsm_adcensus.h declares.

No compute calls here (no GPU in the CPU suite); without a device the product must fail
loudly rather than fall back to a CPU path.
"""
import ctypes
import re

import pytest

import tea_stereo_matching_amd as tsm
from tea_stereo_matching_amd import _native as N


def declared_symbols(path=None):
    text = open(path or N.HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tsm_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_reference_surface():
    syms = declared_symbols()
    for s in ("tsm_adc_create", "tsm_adc_destroy", "tsm_adc_set_disparity_range",
              "tsm_adc_set_strategy", "tsm_adc_set_offset", "tsm_adc_compute",
              "tsm_adc_compute_batch", "tsm_adc_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = N.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # and the binding table covers the whole header
    assert set(declared_symbols()) == set(N.SIGNATURES)


def test_library_exports_every_stereo_ops_symbol():
    lib = N.load()
    syms = declared_symbols(N.OPS_HEADER_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(N.OPS_SIGNATURES)


def test_stereo_ops_argument_errors_without_compute():
    lib = N.load()
    assert lib.tsm_jet_colormap(None) == N.TSM_ERR_ARGUMENT
    assert lib.tsm_apply_colormap(None, 4, 4, 16, None, 0, 0.0, 0.0, None, 12) == N.TSM_ERR_ARGUMENT
    assert lib.tsm_reproject_to_depth_device(None, 4, 4, 16, 1.0, 1.0, None, 16, None) == N.TSM_ERR_ARGUMENT
    assert lib.tsm_remap_linear_fixed_device(None, 4, 4, 12, 3, None, 16, None, 8, 4, 4, None, 12,
                                             None) == N.TSM_ERR_ARGUMENT
    assert lib.tsm_write_point_cloud_pcd(None, 0, None, 0, 0, 0, b"x.pcd") == N.TSM_ERR_ARGUMENT


def test_version_and_device_count():
    assert "gfx950" in tsm.version()
    assert tsm.device_count() >= 0


def test_no_device_fails_loudly():
    if tsm.device_count() > 0:
        pytest.skip("a HIP device is visible")
    lib = N.load()
    h = ctypes.c_void_p()
    assert lib.tsm_adc_create(0, ctypes.byref(h)) == N.TSM_ERR_DEVICE
    with pytest.raises(RuntimeError, match="no usable HIP device"):
        tsm.ADCensus()


def test_null_handle_is_rejected():
    lib = N.load()
    assert lib.tsm_adc_set_offset(None, 1) == N.TSM_ERR_ARGUMENT
    assert lib.tsm_adc_set_disparity_range(None, 0, 10) == N.TSM_ERR_ARGUMENT
    assert lib.tsm_adc_destroy(None) == N.TSM_ERR_ARGUMENT
    assert lib.tsm_adc_last_error(None) == b"null handle"


def test_stereo_header_mirrors_reference_class():
    import os
    text = open(os.path.join(os.path.dirname(N.HEADER_PATH), "stereo.h")).read()
    for s in ("class StereoMatching", "class ADCensus : public StereoMatching",
              "void setMinMaxDisparity(const int& minDisparity, const int& maxDisparity)",
              "void setMatchingStrategy(const ColorModel& colorModel = ColorModel::RGB",
              "void setOffset(const int& offset)", "enum class ColorModel { RGB = 0, HSI = 1 }"):
        assert s in text, s
