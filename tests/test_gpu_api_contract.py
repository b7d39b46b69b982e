"""C-ABI contract on a real MI355X: unsupported parameters are refused (never silently
computed differently from the reference), device calls on caller streams are ordered
against the handle's workspace, and batch errors return without faulting.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tsm():
    import tea_stereo_matching_amd as T

    if T.device_count() == 0:
        pytest.fail("no HIP device visible to a -m gpu test")
    return T


class _Hip:
    """Device buffers and streams through the HIP runtime the library links (torch's
    bundled runtime would be a second, separate device context in this process)."""

    def __init__(self):
        self.rt = ctypes.CDLL("libamdhip64.so.7")
        self.bufs, self.streams = [], []

    def put(self, a: np.ndarray) -> int:
        p = ctypes.c_void_p()
        assert self.rt.hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(a.nbytes, 1))) == 0
        self.bufs.append(p)
        assert self.rt.hipMemcpy(p, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes), 1) == 0
        return p.value

    def get(self, p: int, like: np.ndarray) -> np.ndarray:
        out = np.empty_like(like)
        assert self.rt.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(p),
                                 ctypes.c_size_t(out.nbytes), 2) == 0
        return out

    def stream(self) -> int:
        s = ctypes.c_void_p()
        assert self.rt.hipStreamCreate(ctypes.byref(s)) == 0
        self.streams.append(s)
        return s.value

    def free(self):
        self.rt.hipDeviceSynchronize()
        for p in self.bufs:
            self.rt.hipFree(p)
        for s in self.streams:
            self.rt.hipStreamDestroy(s)


@pytest.fixture()
def hip():
    h = _Hip()
    yield h
    h.free()


@pytest.fixture()
def matcher(tsm):
    m = tsm.ADCensus(0)
    yield m
    m.close()


def test_hsi_custom_lambdas_refused_for_every_census_window(matcher, tsm):
    """ADCensus.cpp:444-451 weights the HSI AD terms by the configured lambdas; the
    device table is exact only for (1, 2.5, 2.5), so any other weights are refused, with
    the 9x7 and with the 7x5 census window alike."""
    left, right = tsm.synthetic.make_scene(3, 32, 48, 9)[:2]
    for win in (0, 1):
        matcher.setMatchingStrategy(tsm.ColorModel.HSI)
        matcher.setMinMaxDisparity(0, 8)
        p = matcher.params()
        p.census_win = win
        p.lambda_hue = 2.0
        matcher.setParams(p)
        with pytest.raises(RuntimeError, match="HSI AD lambdas"):
            matcher.compute(left, right)
    # the default weights still run
    matcher.setMatchingStrategy(tsm.ColorModel.HSI)
    matcher.setMinMaxDisparity(0, 8)
    assert matcher.compute(left, right).shape == (32, 48)


@pytest.mark.parametrize("field", ["blur_kernel_size", "canny_kernel_size"])
def test_non_3x3_blur_and_canny_apertures_refused(matcher, tsm, field):
    """k_eq_blur / k_sobel are cv::blur / cv::Canny with the 3x3 aperture the reference
    configures (stereo_utils.cpp:271-326, ADCensus.cpp:1263-1264); other sizes are refused
    at set time and the previous parameter set stays."""
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    p = matcher.params()
    setattr(p, field, 5)
    with pytest.raises(RuntimeError, match=field):
        matcher.setParams(p)
    assert getattr(matcher.params(), field) == 3


def test_device_calls_on_two_streams_then_host(matcher, tsm, hip):
    """Two tsm_adc_compute_device calls on two caller streams plus a host compute all
    share the handle's first workspace; each result must equal a lone host compute."""
    H, W, mx = 48, 80, 24
    pairs = [tsm.synthetic.make_scene(200 + i, H, W, mx + 1)[:2] for i in range(3)]
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    matcher.setMinMaxDisparity(0, mx)
    matcher.setOmpEmulation(0)
    expect = [matcher.compute(l, r) for l, r in pairs]

    init = np.full((H, W), -7.0, np.float32)
    dl = [hip.put(np.ascontiguousarray(p[0])) for p in pairs[:2]]
    dr = [hip.put(np.ascontiguousarray(p[1])) for p in pairs[:2]]
    outs = [hip.put(init) for _ in range(2)]
    streams = [hip.stream(), hip.stream()]
    for i, s in enumerate(streams):
        matcher.compute_device_ptr(dl[i], dr[i], H, W, W * 3, outs[i], W * 4, s)
    host = matcher.compute(*pairs[2])      # same workspace, the handle's own stream
    matcher.synchronize()                  # waits for both caller streams' pipelines
    assert np.array_equal(host, expect[2])
    for i in range(2):
        assert np.array_equal(hip.get(outs[i], init), expect[i])


def test_batch_device_rejects_null_or_short_output(matcher, tsm, hip):
    """tsm_adc_compute_batch_device checks every output pointer and its row step before
    enqueueing (a bad one is TSM_ERR_ARGUMENT, not a device fault)."""
    from tea_stereo_matching_amd import _native as N

    H, W = 32, 48
    l, r = tsm.synthetic.make_scene(9, H, W, 9)[:2]
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    matcher.setMinMaxDisparity(0, 8)
    init = np.zeros((H, W), np.float32)
    dl, dr, out = hip.put(np.ascontiguousarray(l)), hip.put(np.ascontiguousarray(r)), hip.put(init)
    lib = N.load()
    h = matcher._h
    lp = (ctypes.c_void_p * 2)(dl, dl)
    rp = (ctypes.c_void_p * 2)(dr, dr)
    op = (ctypes.c_void_p * 2)(out, None)
    assert lib.tsm_adc_compute_batch_device(h, 2, lp, rp, H, W, W * 3, op, W * 4) == N.TSM_ERR_ARGUMENT
    assert b"output buffer" in lib.tsm_adc_last_error(h)
    op = (ctypes.c_void_p * 2)(out, out)
    assert lib.tsm_adc_compute_batch_device(h, 2, lp, rp, H, W, W * 3, op, W * 4 - 4) == N.TSM_ERR_ARGUMENT
    # the handle stays usable
    assert lib.tsm_adc_compute_batch_device(h, 2, lp, rp, H, W, W * 3, op, W * 4) == N.TSM_OK
    assert np.array_equal(hip.get(out, init), matcher.compute(l, r))


def test_batch_host_error_midway_drains_queued_pairs(matcher, tsm):
    """An invalid pair inside tsm_adc_compute_batch returns its error after the groups
    already enqueued have finished (their host buffers are safe to free): with groups of
    two, pairs 0-1 run as the first group and the second group (pair 2) is refused."""
    H, W = 40, 64
    pairs = [tsm.synthetic.make_scene(300 + i, H, W, 17)[:2] for i in range(3)]
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    matcher.setMinMaxDisparity(0, 16)
    matcher.setConcurrency(2)
    from tea_stereo_matching_amd import _native as N

    lib = N.load()
    outs = [np.full((H, W), -7.0, np.float32) for _ in range(3)]
    ls = [np.ascontiguousarray(p[0]) for p in pairs]
    rs = [np.ascontiguousarray(p[1]) for p in pairs]
    lp = (ctypes.c_void_p * 3)(ls[0].ctypes.data, ls[1].ctypes.data, None)  # third pair invalid
    rp = (ctypes.c_void_p * 3)(*[x.ctypes.data for x in rs])
    op = (ctypes.c_void_p * 3)(*[x.ctypes.data for x in outs])
    rc = lib.tsm_adc_compute_batch(matcher._h, 3, lp, rp, H, W, W * 3, op, W * 4)
    assert rc == N.TSM_ERR_IMAGE
    # the first two pairs completed before the call returned
    for i in range(2):
        assert np.array_equal(outs[i], matcher.compute(*pairs[i]))


def test_host_paths_with_padded_row_steps(matcher, tsm):
    """Host images and outputs with row steps wider than the row (cv::Mat ROIs): the
    pinned staging copies row by row, through the single call and a batch of groups that
    reuse a workspace (5 pairs in groups of 2 over two workspaces)."""
    from tea_stereo_matching_amd import _native as N

    H, W, pad_in, pad_out = 36, 70, 13, 5
    pairs = [tsm.synthetic.make_scene(400 + i, H, W, 17)[:2] for i in range(5)]
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    matcher.setMinMaxDisparity(0, 16)
    matcher.setConcurrency(2)
    want = [matcher.compute(l, r) for l, r in pairs]
    step, ostep = W * 3 + pad_in, W * 4 + 4 * pad_out
    bl = [np.zeros((H, step), np.uint8) for _ in pairs]
    br = [np.zeros((H, step), np.uint8) for _ in pairs]
    for i, (l, r) in enumerate(pairs):
        bl[i][:, :W * 3] = l.reshape(H, W * 3)
        br[i][:, :W * 3] = r.reshape(H, W * 3)
    outs = [np.full((H, W + pad_out), -7.0, np.float32) for _ in pairs]
    lib = N.load()
    lp = (ctypes.c_void_p * 5)(*[x.ctypes.data for x in bl])
    rp = (ctypes.c_void_p * 5)(*[x.ctypes.data for x in br])
    op = (ctypes.c_void_p * 5)(*[x.ctypes.data for x in outs])
    assert lib.tsm_adc_compute_batch(matcher._h, 5, lp, rp, H, W, step, op, ostep) == 0
    for i in range(5):
        assert np.array_equal(outs[i][:, :W], want[i])
        assert np.all(outs[i][:, W:] == -7.0)  # the padding of each output row is untouched
    one = np.full((H, W + pad_out), -7.0, np.float32)
    assert lib.tsm_adc_compute(matcher._h, bl[3].ctypes.data, br[3].ctypes.data, H, W, step,
                               one.ctypes.data, ostep) == 0
    assert np.array_equal(one[:, :W], want[3]) and np.all(one[:, W:] == -7.0)
