"""The operators either side of the AD-Census path, mirroring the
reference's free functions in namespace stereo (include/stereo.h, source/stereo.cpp) and
its EpipolarRectify class (source/EpipolarRectify.cpp), over the gfx950 kernels of
libtsm_adcensus.so (include/tsm_stereo_ops.h).

numpy arrays go through the host entry points (synchronous); torch tensors on a HIP
device go through the _device entry points and the results stay on the device.  torch
bundles its own HIP runtime, whose streams the library's runtime cannot use, so a
device call waits for torch's current stream, runs on the library's null stream and
waits for it (synchronous too).  There is no CPU fallback: without the library or a
device the calls raise.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _native as N


def _check(rc: int, what: str) -> None:
    if rc == N.TSM_OK:
        return
    if rc == N.TSM_ERR_ARGUMENT:
        raise ValueError(f"{what}: invalid argument")
    raise RuntimeError(f"{what}: status {rc}")


def _is_dev(a) -> bool:
    return getattr(a, "is_cuda", False)


def _stream():
    """Order a _device call after torch's pending work (see the module docstring)."""
    import torch

    torch.cuda.current_stream().synchronize()
    return None


def _done(rc: int, dev: bool) -> int:
    if dev and rc == N.TSM_OK:
        rc = N.load().tsm_stream_synchronize(None)
    return rc


def _ptr(a):
    if _is_dev(a):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    if _is_dev(a):
        import torch

        if a.dtype != torch.float32 or a.dim() != 2:
            raise ValueError(f"expected a 2-D float32 tensor, got {a.dtype} with {a.dim()} dims")
        return a.contiguous()
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 2:
        raise ValueError(f"expected a 2-D float32 map, got {a.ndim} dims")
    return a


def _empty_like(ref, shape, dtype):
    if _is_dev(ref):
        import torch

        tdt = {np.uint8: torch.uint8, np.float32: torch.float32}[dtype]
        return torch.empty(shape, dtype=tdt, device=ref.device)
    return np.zeros(shape, dtype)


# ---- f2 ------------------------------------------------------------------------------

def JETColorMap() -> np.ndarray:
    """stereo::JETColorMap (stereo.cpp:75-92): a 1 x 256 BGR table."""
    lut = np.zeros((1, 256, 3), np.uint8)
    _check(N.load().tsm_jet_colormap(_ptr(lut)), "JETColorMap")
    return lut


def applyColorMap(src, *args):
    """applyColorMap(src, colorMap) (stereo.cpp:94-118) or
    applyColorMap(src, minVal, maxVal, colorMap) (stereo.cpp:120-134); returns dst."""
    if len(args) == 1:
        (cmap,), use_range, mn, mx = args, 0, 0.0, 0.0
    elif len(args) == 3:
        mn, mx, cmap = args
        use_range = 1
    else:
        raise TypeError("applyColorMap(src, colorMap) or applyColorMap(src, minVal, maxVal, colorMap)")
    lut = np.ascontiguousarray(np.asarray(cmap, dtype=np.uint8).reshape(256, 3))
    s = _f32(src)
    H, W = s.shape
    dst = _empty_like(s, (H, W, 3), np.uint8)
    lib = N.load()
    if _is_dev(s):
        rc = lib.tsm_apply_colormap_device(_ptr(s), H, W, 4 * W, _ptr(lut), use_range, float(mn),
                                           float(mx), _ptr(dst), 3 * W, _stream())
    else:
        rc = lib.tsm_apply_colormap(_ptr(s), H, W, 4 * W, _ptr(lut), use_range, float(mn), float(mx),
                                    _ptr(dst), 3 * W)
    _check(_done(rc, _is_dev(s)), "applyColorMap")
    return dst


# ---- f3 ------------------------------------------------------------------------------

def reprojectToDepth(disparity, focalLength: float, baseline: float):
    """stereo::reprojectToDepth (stereo.cpp:136-148)."""
    s = _f32(disparity)
    H, W = s.shape
    dst = _empty_like(s, (H, W), np.float32)
    lib = N.load()
    if _is_dev(s):
        rc = lib.tsm_reproject_to_depth_device(_ptr(s), H, W, 4 * W, focalLength, baseline, _ptr(dst),
                                               4 * W, _stream())
    else:
        rc = lib.tsm_reproject_to_depth(_ptr(s), H, W, 4 * W, focalLength, baseline, _ptr(dst), 4 * W)
    _check(_done(rc, _is_dev(s)), "reprojectToDepth")
    return dst


def reprojectTo3D(disparity, *args):
    """reprojectTo3D(disparity, focalLength, baseline, cx, cy) (stereo.cpp:150-169) or
    reprojectTo3D(disparity, Q) (stereo.cpp:171-202); returns H x W x 3 fp32 points."""
    s = _f32(disparity)
    H, W = s.shape
    dst = _empty_like(s, (H, W, 3), np.float32)
    lib = N.load()
    dev = _is_dev(s)
    if len(args) == 4:
        f, b, cx, cy = (float(v) for v in args)
        rc = (lib.tsm_reproject_to_3d_device(_ptr(s), H, W, 4 * W, f, b, cx, cy, _ptr(dst), 12 * W, _stream())
              if dev else lib.tsm_reproject_to_3d(_ptr(s), H, W, 4 * W, f, b, cx, cy, _ptr(dst), 12 * W))
    elif len(args) == 1:
        q = np.ascontiguousarray(np.asarray(args[0], dtype=np.float64).reshape(16))
        rc = (lib.tsm_reproject_to_3d_q_device(_ptr(s), H, W, 4 * W, _ptr(q), _ptr(dst), 12 * W, _stream())
              if dev else lib.tsm_reproject_to_3d_q(_ptr(s), H, W, 4 * W, _ptr(q), _ptr(dst), 12 * W))
    else:
        raise TypeError("reprojectTo3D(disparity, f, b, cx, cy) or reprojectTo3D(disparity, Q)")
    _check(_done(rc, dev), "reprojectTo3D")
    return dst


def _write_cloud(fn: str, RGBImage, XYZPoints, path: str) -> None:
    img = np.ascontiguousarray(np.asarray(RGBImage, dtype=np.uint8))
    xyz = np.ascontiguousarray(np.asarray(XYZPoints, dtype=np.float32))
    if img.size == 0 or xyz.size == 0 or not path:
        return  # the reference logs "Empty input." and returns (stereo.cpp:252-256)
    if xyz.ndim != 3 or xyz.shape[2] != 3 or img.ndim != 3 or img.shape != xyz.shape[:2] + (3,):
        raise ValueError(f"{fn}: expected H x W x 3 BGR image and points of one size, got "
                         f"{img.shape} and {xyz.shape}")
    H, W = xyz.shape[:2]
    rc = getattr(N.load(), fn)(_ptr(img), 3 * W, _ptr(xyz), 12 * W, H, W, path.encode())
    _check(rc, fn)


def writePointCloudToPCD(RGBImage, XYZPoints, pcdPath: str) -> None:
    """stereo::writePointCloudToPCD (stereo.cpp:250-278); RGBImage is BGR-ordered."""
    _write_cloud("tsm_write_point_cloud_pcd", RGBImage, XYZPoints, pcdPath)


def writePointCloudToPLY(RGBImage, XYZPoints, plyPath: str) -> None:
    """stereo::writePointCloudToPLY (stereo.cpp:328-356)."""
    _write_cloud("tsm_write_point_cloud_ply", RGBImage, XYZPoints, plyPath)


# ---- f4 ------------------------------------------------------------------------------

def remap(src, map1, map2):
    """cv::remap(src, dst, map1, map2, INTER_LINEAR) with BORDER_CONSTANT 0: map1/map2 either
    int16 H x W x 2 + uint16 H x W (CV_16SC2 + CV_16UC1) or float32 x / y maps."""
    dev = _is_dev(src)
    lib = N.load()
    if dev:
        import torch

        src = src.contiguous()
        C = 1 if src.dim() == 2 else src.shape[2]
        fixed = map1.dtype == torch.int16
    else:
        src = np.ascontiguousarray(src, dtype=np.uint8)
        C = 1 if src.ndim == 2 else src.shape[2]
        fixed = np.asarray(map1).dtype == np.int16
    sh, sw = src.shape[:2]
    if fixed:
        m1 = map1.contiguous() if dev else np.ascontiguousarray(map1, dtype=np.int16)
        m2 = map2.contiguous() if dev else np.ascontiguousarray(map2, dtype=np.uint16)
        H, W = m2.shape
        dst = _empty_like(src, (H, W, C) if C > 1 else (H, W), np.uint8)
        args = (_ptr(src), sh, sw, C * sw, C, _ptr(m1), 4 * W, _ptr(m2), 2 * W, H, W, _ptr(dst), C * W)
        rc = (lib.tsm_remap_linear_fixed_device(*args, _stream()) if dev else lib.tsm_remap_linear_fixed(*args))
    else:
        m1, m2 = _f32(map1), _f32(map2)
        H, W = m1.shape
        dst = _empty_like(src, (H, W, C) if C > 1 else (H, W), np.uint8)
        args = (_ptr(src), sh, sw, C * sw, C, _ptr(m1), _ptr(m2), 4 * W, H, W, _ptr(dst), C * W)
        rc = (lib.tsm_remap_linear_float_device(*args, _stream()) if dev else lib.tsm_remap_linear_float(*args))
    _check(_done(rc, dev), "remap")
    return dst


# ---- group forms (device tensors): a batch's maps through one launch per 64 ----------

def _ptr_array(ts):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def _dev_batch(srcs, what):
    srcs = [t.contiguous() for t in srcs]
    if not srcs or not all(_is_dev(t) for t in srcs) or len({tuple(t.shape) for t in srcs}) != 1:
        raise ValueError(f"{what}: expected a non-empty list of device tensors of one shape")
    return srcs


def applyColorMapBatch(disparities, *args):
    """applyColorMap over a list of (H, W) float32 device tensors (tsm_apply_colormap_batch_device),
    with applyColorMap's argument forms: (disparities, colorMap) or (disparities, minVal,
    maxVal, colorMap); (disparities) alone uses JETColorMap().  Per map the same image as
    applyColorMap; returns a list of (H, W, 3) uint8 tensors."""
    import torch

    if len(args) == 3 and (_is_dev(args[0]) or isinstance(args[0], np.ndarray)) and np.ndim(args[2]) == 0:
        # the round-3 form (disparities, colorMap, minVal, maxVal): refuse it by name
        raise TypeError("applyColorMapBatch takes applyColorMap's order: (disparities, minVal, maxVal, colorMap)")
    if len(args) == 0:
        cmap, use_range, mn, mx = JETColorMap(), 0, 0.0, 0.0
    elif len(args) == 1:
        (cmap,), use_range, mn, mx = args, 0, 0.0, 0.0
    elif len(args) == 3:
        mn, mx, cmap = args
        if mn is None or mx is None:
            raise ValueError("applyColorMapBatch: minVal and maxVal must both be given")
        use_range = 1
    else:
        raise TypeError("applyColorMapBatch(disparities[, colorMap]) or "
                        "applyColorMapBatch(disparities, minVal, maxVal, colorMap)")
    ss = _dev_batch([_f32(d) for d in disparities], "applyColorMapBatch")
    H, W = ss[0].shape
    lut = np.ascontiguousarray(np.asarray(cmap, dtype=np.uint8).reshape(256, 3))
    outs = [torch.empty((H, W, 3), dtype=torch.uint8, device=ss[0].device) for _ in ss]
    rc = N.load().tsm_apply_colormap_batch_device(len(ss), _ptr_array(ss), H, W, 4 * W, _ptr(lut), use_range,
                                                  float(mn), float(mx), _ptr_array(outs), 3 * W, _stream())
    _check(_done(rc, True), "applyColorMapBatch")
    return outs


def reprojectToDepthBatch(disparities, focalLength: float, baseline: float):
    """reprojectToDepth over a list of device tensors (tsm_reproject_to_depth_batch_device)."""
    import torch

    ss = _dev_batch([_f32(d) for d in disparities], "reprojectToDepthBatch")
    H, W = ss[0].shape
    outs = [torch.empty((H, W), dtype=torch.float32, device=ss[0].device) for _ in ss]
    rc = N.load().tsm_reproject_to_depth_batch_device(len(ss), _ptr_array(ss), H, W, 4 * W, focalLength, baseline,
                                                      _ptr_array(outs), 4 * W, _stream())
    _check(_done(rc, True), "reprojectToDepthBatch")
    return outs


def reprojectTo3DBatch(disparities, focalLength: float, baseline: float, cx: float, cy: float):
    """reprojectTo3D(d, f, b, cx, cy) over a list of device tensors (tsm_reproject_to_3d_batch_device)."""
    import torch

    ss = _dev_batch([_f32(d) for d in disparities], "reprojectTo3DBatch")
    H, W = ss[0].shape
    outs = [torch.empty((H, W, 3), dtype=torch.float32, device=ss[0].device) for _ in ss]
    rc = N.load().tsm_reproject_to_3d_batch_device(len(ss), _ptr_array(ss), H, W, 4 * W, focalLength, baseline, cx,
                                                   cy, _ptr_array(outs), 12 * W, _stream())
    _check(_done(rc, True), "reprojectTo3DBatch")
    return outs


def remapBatch(srcs, map1, map2):
    """cv::remap INTER_LINEAR of a list of uint8 device images of one size through the same
    CV_16SC2 + CV_16UC1 maps (tsm_remap_linear_fixed_batch_device): map1 int16 (H, W, 2),
    map2 uint16/int16 (H, W), both on the images' device.  Float maps go through remap()."""
    import torch

    ss = _dev_batch(srcs, "remapBatch")
    if ss[0].dtype != torch.uint8 or ss[0].dim() not in (2, 3):
        raise ValueError("remapBatch: sources must be uint8 (H, W) or (H, W, C) device tensors")
    if not (_is_dev(map1) and _is_dev(map2)) or map1.device != ss[0].device or map2.device != ss[0].device:
        raise ValueError("remapBatch: map1 and map2 must be tensors on the sources' device")
    if map1.dtype != torch.int16 or map2.dtype not in (torch.uint16, torch.int16):
        raise ValueError("remapBatch: expects CV_16SC2 (int16) + CV_16UC1 (uint16) maps; "
                         "use remap() for float32 maps")
    if map1.dim() != 3 or map1.shape[2] != 2 or map2.dim() != 2 or tuple(map1.shape[:2]) != tuple(map2.shape):
        raise ValueError("remapBatch: map1 must be (H, W, 2) and map2 (H, W) of the same H, W")
    C = 1 if ss[0].dim() == 2 else ss[0].shape[2]
    sh, sw = ss[0].shape[:2]
    m1, m2 = map1.contiguous(), map2.contiguous()
    H, W = m2.shape
    outs = [torch.empty((H, W, C) if C > 1 else (H, W), dtype=torch.uint8, device=ss[0].device) for _ in ss]
    rc = N.load().tsm_remap_linear_fixed_batch_device(len(ss), _ptr_array(ss), sh, sw, C * sw, C, _ptr(m1), 4 * W,
                                                      _ptr(m2), 2 * W, H, W, _ptr_array(outs), C * W, _stream())
    _check(_done(rc, True), "remapBatch")
    return outs


@dataclass
class EpipolarRectifyMap:
    """stereo::EpipolarRectifyMap (stereo_utils.h / stereo_utils.cpp:88-174): rectification
    rotations / projections and the two remap map pairs of each camera."""

    R1: np.ndarray | None = None
    R2: np.ndarray | None = None
    P1: np.ndarray | None = None
    P2: np.ndarray | None = None
    map00: object = None
    map01: object = None
    map10: object = None
    map11: object = None

    def empty(self) -> bool:  # stereo_utils.cpp:171-174
        return any(m is None or getattr(m, "size", 0) == 0 or (hasattr(m, "numel") and m.numel() == 0)
                   for m in (self.map00, self.map01, self.map10, self.map11))


class EpipolarRectify:
    """stereo::EpipolarRectify (stereo.h:254-296, EpipolarRectify.cpp)."""

    def __init__(self, rectifyMap: EpipolarRectifyMap | None = None, imgsz=None):
        self._map = EpipolarRectifyMap()
        self._imgsz = None
        if rectifyMap is not None:
            self.loadEpipolarRectifyMap(rectifyMap, imgsz)

    def loadEpipolarRectifyMap(self, rectifyMap: EpipolarRectifyMap, imgsz) -> None:
        """EpipolarRectify.cpp:32-44; imgsz = (width, height) as cv::Size."""
        if rectifyMap is None or rectifyMap.empty():
            raise RuntimeError("stereo params is empty, please load it first")
        self._map = rectifyMap
        self._imgsz = tuple(imgsz) if imgsz is not None else None

    def rectify(self, *images, split: bool = False):
        """rectify(stereoImage) -> side-by-side rectified image (EpipolarRectify.cpp:46-64),
        rectify(stereoImage, split=True) -> (left, right) (:66-82),
        rectify(left, right) -> (left, right) (:84-101).  Returns None where the reference
        logs an error and returns (maps not loaded, empty image)."""
        if self._map.empty():
            return None
        if len(images) == 1:
            img = images[0]
            if img is None or (getattr(img, "size", 0) == 0 and not _is_dev(img)):
                return None
            w, h = self._imgsz
            left, right = img[:h, :w], img[:h, w:2 * w]
            l, r = self._rectify_pair(left, right)
            if split:
                return l, r
            if _is_dev(l):
                import torch

                return torch.cat([l, r], dim=1)
            return np.concatenate([l, r], axis=1)
        if len(images) == 2:
            left, right = images
            if left is None or right is None:
                return None
            return self._rectify_pair(left, right)
        raise TypeError("rectify(stereoImage) or rectify(left, right)")

    def _rectify_pair(self, left, right):
        m = self._map
        return remap(left, m.map00, m.map01), remap(right, m.map10, m.map11)
