"""stereo::ADCensus for Python, over the MI355X C ABI (include/tsm_adcensus.h).

Mirrors the reference class (YYpasser/tea_stereo_matching include/stereo.h:388-422,
source/ADCensus.cpp): same method names, argument meaning and error behaviour.  The
reference throws ``std::string`` from the setters and the input check; here those become
:class:`ADCensusError` with the identical message, and internal failures become
``RuntimeError`` (ADCensus.cpp:383-387 rethrows as ``std::runtime_error``).

Images are ``(H, W, 3) uint8`` BGR arrays (cv::Mat CV_8UC3); ``compute`` returns the
``(H, W) float32`` disparity of the left view (CV_32FC1).
"""
from __future__ import annotations

import ctypes
from enum import IntEnum
from typing import Sequence

import numpy as np

from . import _native as N


class ColorModel(IntEnum):
    """stereo_utils.h:191-195"""

    RGB = 0
    HSI = 1


class CensusWin(IntEnum):
    """stereo_utils.h:200-204"""

    CENSUSWIN_9x7 = 0
    CENSUSWIN_7x5 = 1


class ADCensusError(Exception):
    """The reference's ``throw(std::string(...))`` (ADCensus.cpp:310, :326, :333)."""


_IMAGE_ERROR = "[ADCensus] Image error."


def _check_image(img) -> np.ndarray:
    if img is None:
        raise ADCensusError(_IMAGE_ERROR)
    a = np.asarray(img)
    if a.size == 0 or a.ndim != 3 or a.shape[2] != 3 or a.dtype != np.uint8:
        raise ADCensusError(_IMAGE_ERROR)
    return np.ascontiguousarray(a)


class ADCensus:
    """AD-Census stereo matcher on one HIP device (default ordinal 0)."""

    def __init__(self, device: int = 0):
        self._lib = N.load()
        h = ctypes.c_void_p()
        rc = self._lib.tsm_adc_create(int(device), ctypes.byref(h))
        if rc != N.TSM_OK:
            raise RuntimeError(
                f"[ADCensus] no usable HIP device {device} (tsm_adc_create returned {rc}); "
                "this matcher runs on MI355X only, there is no CPU path")
        self._h = h
        self.device = int(device)
        self._roi_or_mask = False

    # -- lifetime -------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.tsm_adc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- errors -----------------------------------------------------------------
    def _raise(self, rc: int):
        msg = (self._lib.tsm_adc_last_error(self._h) or b"").decode()
        if rc in (N.TSM_ERR_DISPARITY_RANGE, N.TSM_ERR_OFFSET, N.TSM_ERR_IMAGE):
            raise ADCensusError(msg)
        raise RuntimeError(msg or f"tsm_adc error {rc}")

    def _ok(self, rc: int):
        if rc != N.TSM_OK:
            self._raise(rc)

    # -- reference API (stereo.h:399-418) -------------------------------------
    def setMinMaxDisparity(self, minDisparity: int, maxDisparity: int) -> None:
        self._ok(self._lib.tsm_adc_set_disparity_range(self._h, int(minDisparity), int(maxDisparity)))

    def setMatchingStrategy(self, colorModel: ColorModel = ColorModel.RGB, roiMatching: bool = False,
                            maskMatching: bool = False) -> None:
        self._ok(self._lib.tsm_adc_set_strategy(self._h, int(colorModel), int(bool(roiMatching)),
                                                int(bool(maskMatching))))
        self._roi_or_mask = bool(roiMatching) or bool(maskMatching)

    def setOffset(self, offset: int) -> None:
        self._ok(self._lib.tsm_adc_set_offset(self._h, int(offset)))

    def compute(self, leftImage, rightImage, disparity: np.ndarray | None = None) -> np.ndarray:
        """Disparity of the left view; writes into ``disparity`` when given (H, W) float32."""
        l, r = _check_image(leftImage), _check_image(rightImage)
        if l.shape != r.shape:
            raise ADCensusError(_IMAGE_ERROR)
        H, W = l.shape[:2]
        out = np.empty((H, W), np.float32)
        self._ok(self._lib.tsm_adc_compute(self._h, l.ctypes.data, r.ctypes.data, H, W, W * 3,
                                           out.ctypes.data, W * 4))
        if disparity is not None:
            disparity[...] = out
            return disparity
        return out

    def compute_batch(self, leftImages: Sequence, rightImages: Sequence) -> list[np.ndarray]:
        """Batch form (ONNXRuntimeInference::compute(vector...), stereo.h:381)."""
        if len(leftImages) != len(rightImages):
            raise ADCensusError(_IMAGE_ERROR)
        ls = [_check_image(x) for x in leftImages]
        rs = [_check_image(x) for x in rightImages]
        if not ls:
            return []
        shape = ls[0].shape
        if any(x.shape != shape for x in ls + rs):
            return [self.compute(a, b) for a, b in zip(ls, rs)]
        H, W = shape[:2]
        outs = [np.empty((H, W), np.float32) for _ in ls]
        n = len(ls)
        lp = (ctypes.c_void_p * n)(*[x.ctypes.data for x in ls])
        rp = (ctypes.c_void_p * n)(*[x.ctypes.data for x in rs])
        op = (ctypes.c_void_p * n)(*[x.ctypes.data for x in outs])
        self._ok(self._lib.tsm_adc_compute_batch(self._h, n, lp, rp, H, W, W * 3, op, W * 4))
        return outs

    # -- device-resident entry points (HBM pointers, e.g. torch tensor data_ptr) ---------
    def compute_device_ptr(self, left_ptr: int, right_ptr: int, rows: int, cols: int, step: int,
                           out_ptr: int, out_step: int, stream: int | None = None) -> None:
        self._ok(self._lib.tsm_adc_compute_device(self._h, left_ptr, right_ptr, rows, cols, step,
                                                  out_ptr, out_step, stream))

    def compute_batch_device_ptr(self, left_ptrs, right_ptrs, rows: int, cols: int, step: int,
                                 out_ptrs, out_step: int) -> None:
        n = len(left_ptrs)
        lp = (ctypes.c_void_p * n)(*left_ptrs)
        rp = (ctypes.c_void_p * n)(*right_ptrs)
        op = (ctypes.c_void_p * n)(*out_ptrs)
        self._ok(self._lib.tsm_adc_compute_batch_device(self._h, n, lp, rp, rows, cols, step, op,
                                                        out_step))

    def synchronize(self) -> None:
        self._ok(self._lib.tsm_adc_synchronize(self._h))

    # -- extensions ------------------------------------------------------------
    def getMinMaxDisparity(self) -> tuple[int, int]:
        a, b = ctypes.c_int(), ctypes.c_int()
        self._ok(self._lib.tsm_adc_get_disparity_range(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def params(self) -> N.TsmParams:
        p = N.TsmParams()
        self._ok(self._lib.tsm_adc_get_params(self._h, ctypes.byref(p)))
        return p

    def setParams(self, p: N.TsmParams) -> None:
        self._ok(self._lib.tsm_adc_set_params(self._h, ctypes.byref(p)))

    def setConcurrency(self, streams: int) -> None:
        self._ok(self._lib.tsm_adc_set_concurrency(self._h, int(streams)))

    def setOmpEmulation(self, threads: int) -> None:
        """Reproduce the reference's racy omp-static scanline outcome for ``threads``."""
        self._ok(self._lib.tsm_adc_set_omp_emulation(self._h, int(threads)))

    def setProfiling(self, enable: bool) -> None:
        self._ok(self._lib.tsm_adc_set_profiling(self._h, int(bool(enable))))

    def stageTimes(self) -> dict[str, tuple[float, int]]:
        ms = (ctypes.c_double * len(N.STAGES))()
        cnt = (ctypes.c_int * len(N.STAGES))()
        self._ok(self._lib.tsm_adc_stage_times(self._h, ms, cnt, len(N.STAGES)))
        return {k: (ms[i], cnt[i]) for i, k in enumerate(N.STAGES)}

    def resetStageTimes(self) -> None:
        self._ok(self._lib.tsm_adc_reset_stage_times(self._h))

    def workspaceBytes(self, rows: int, cols: int) -> int:
        """HBM bytes of one pair slot (a batch handle holds 2 x concurrency of them)."""
        return int(self._lib.tsm_adc_workspace_bytes(self._h, rows, cols))

    def convert_hsi(self, image) -> np.ndarray:
        """bgr2hsi on the device (ADCensus.cpp:1429-1473) as the current strategy runs it:
        with the hue-band filter in ROI / mask mode (:1463-1470).  (H, W, 3) H S I bytes."""
        a = _check_image(image)
        H, W = a.shape[:2]
        out = np.empty_like(a)
        filt = int(self._roi_or_mask)
        self._ok(self._lib.tsm_adc_convert_hsi(self._h, a.ctypes.data, H, W, W * 3, filt, out.ctypes.data, W * 3))
        return out

    def compute_debug(self, leftImage, rightImage, stages=()) -> tuple[np.ndarray, dict]:
        """compute() plus per-stage dumps in the reference layout (tsm_adc_dump)."""
        l, r = _check_image(leftImage), _check_image(rightImage)
        if l.shape != r.shape:
            raise ADCensusError(_IMAGE_ERROR)
        H, W = l.shape[:2]
        mn, mx = self.getMinMaxDisparity()
        L = mx - mn + 1
        shapes = {
            "images": ((2, H, W, 3), np.uint8), "cost_init": ((2, L, H, W), np.float32),
            "arms": ((2, 4, H, W), np.int32), "cost_agg": ((2, L, H, W), np.float32),
            "cost_scan": ((2, L, H, W), np.float32), "wta": ((2, H, W), np.int32),
            "outlier": ((H, W), np.int32), "voting": ((H, W), np.int32),
            "interp": ((H, W), np.int32), "gray": ((H, W), np.uint8),
            "edges": ((H, W), np.uint8), "adjusted": ((H, W), np.int32),
            "subpix": ((H, W), np.float32),
        }
        dumps = {k: np.zeros(*shapes[k]) for k in stages}
        d = N.TsmDump(**{k: v.ctypes.data for k, v in dumps.items()})
        out = np.empty((H, W), np.float32)
        self._ok(self._lib.tsm_adc_compute_debug(self._h, l.ctypes.data, r.ctypes.data, H, W, W * 3,
                                                 out.ctypes.data, W * 4, ctypes.byref(d)))
        return out, dumps
