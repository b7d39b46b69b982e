"""tea_stereo_matching_amd -- MI355X-native AD-Census stereo matcher.

Drop-in for the one hot path of YYpasser/tea_stereo_matching, ``stereo::ADCensus``
(include/stereo.h:388-422, source/ADCensus.cpp): hand-written gfx950 HIP kernels behind
the C ABI in ``include/tsm_adcensus.h``; this package is the Python mirror of the
reference class plus the synthetic-pair generator used by the benchmark.
"""
from .adcensus import ADCensus, ADCensusError, CensusWin, ColorModel  # noqa: F401
from ._native import LIB_PATH, device_count, version  # noqa: F401
from . import synthetic  # noqa: F401
from .stereo_ops import (EpipolarRectify, EpipolarRectifyMap, JETColorMap, applyColorMap,  # noqa: F401
                         applyColorMapBatch, remap, remapBatch, reprojectTo3D, reprojectTo3DBatch,
                         reprojectToDepth, reprojectToDepthBatch, writePointCloudToPCD,
                         writePointCloudToPLY)

__all__ = ["ADCensus", "ADCensusError", "CensusWin", "ColorModel", "LIB_PATH", "device_count",
           "version", "synthetic"]
