"""HIP path vs the oracle (CPU restatement of source/ADCensus.cpp), on a real MI355X.

Bar: bit-exact.  Census, arms, WTA/outlier/voting/interpolation maps are integers; the
cost volumes are fp32 computed in the reference's exact operation order (sequential arm
sums, host-built expf tables, no FMA contraction), so every stage is compared with
np.array_equal -- including the final float disparity.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, host_threads, load_bgr

pytestmark = pytest.mark.gpu

STAGES = ("images", "cost_init", "arms", "cost_agg", "cost_scan", "wta", "outlier", "voting",
          "interp", "gray", "edges", "adjusted", "subpix")


@pytest.fixture(scope="module")
def tsm():
    import tea_stereo_matching_amd as T

    if T.device_count() == 0:
        pytest.fail("no HIP device visible to a -m gpu test")
    return T


@pytest.fixture(scope="module")
def matcher(tsm):
    m = tsm.ADCensus(0)
    yield m
    m.close()


def _oracle_params(oracle, model, mn, mx, **kw):
    return oracle.default_params(model, mn, mx, num_threads=host_threads(), **kw)


def _gpu(matcher, tsm, left, right, model, mn, mx, stages=(), omp=0, roi=False, mask=False):
    matcher.setMatchingStrategy(tsm.ColorModel(model), roi, mask)
    matcher.setMinMaxDisparity(mn, mx)
    matcher.setOmpEmulation(omp)
    if stages:
        return matcher.compute_debug(left, right, stages)
    return matcher.compute(left, right), {}


def _assert_stages_equal(g, o, stages):
    for s in stages:
        a, b = g[s], o[s]
        if s == "cost_scan":  # the GPU keeps both views only in debug runs; compare both
            pass
        if not np.array_equal(a, b):
            diff = np.argwhere(a != b) if a.shape == b.shape else None
            n = 0 if diff is None else len(diff)
            first = None if diff is None or not n else tuple(diff[0])
            pytest.fail(f"stage {s}: {n} mismatches (shape {a.shape} vs {b.shape}), first at {first}"
                        + ("" if first is None else f": gpu={a[first]} oracle={b[first]}"))


def _synthetic(tsm, seed, H, W, L):
    return tsm.synthetic.make_scene(seed, H, W, L)[:2]


CASES = [
    # (seed, H, W, minD, maxD)
    (1, 64, 96, 0, 24),
    (2, 120, 160, 0, 48),
    (3, 97, 131, 0, 64),     # odd sizes, L=65 (Lp padding)
    (4, 80, 120, 5, 40),     # minD > 0 (reference index quirks, :556-561, :1398)
    (5, 48, 64, 0, 40),      # D >= W/2
]


@pytest.mark.parametrize("case", CASES, ids=[f"s{c[0]}_{c[1]}x{c[2]}_d{c[3]}-{c[4]}" for c in CASES])
def test_stages_bit_exact_synthetic(matcher, tsm, oracle, case):
    seed, H, W, mn, mx = case
    left, right = _synthetic(tsm, seed, H, W, mx - mn + 1)
    d_g, g = _gpu(matcher, tsm, left, right, 0, mn, mx, STAGES)
    d_o, o = oracle.compute(left, right, _oracle_params(oracle, oracle.RGB, mn, mx), STAGES)
    _assert_stages_equal(g, o, STAGES)
    assert np.array_equal(d_g, d_o)


WIDE = [
    # (seed, H, W, minD, maxD, model): the three-labels-a-lane walk (Lp 192 / 196) and its
    # tail float4 (labels 192..195), both views, RGB and HSI
    (31, 24, 300, 0, 192, 0),
    (32, 20, 270, 0, 191, 0),
    (33, 20, 270, 0, 188, 0),
    (34, 22, 290, 0, 192, 1),
    (35, 18, 260, 3, 195, 0),
    # past 256 labels (configs C and E): four / five labels a lane + the tail float4 in the
    # cost walk, two label vectors a lane in the scanline and the aggregation
    (36, 24, 300, 0, 256, 0),
    (37, 20, 340, 0, 320, 0),
    (38, 22, 310, 0, 256, 1),
    (39, 20, 300, 0, 258, 0),   # tail float4 with three real labels (257..259)
    (40, 18, 360, 0, 323, 0),   # E = 5 lanes + a full tail (labels 320..323)
    # every other range setMinMaxDisparity accepts: eight labels a lane (and label slices of
    # 512 past Lp 512) in the cost walk; the split streamer in as many label slices as keep
    # its rings inside the CU's LDS; the scanline's 2 / 3 / 4 / 8 label vectors a lane
    (48, 20, 300, 0, 240, 0),   # Lp 244: four labels a lane, two aggregation slices
    (41, 16, 300, 0, 264, 0),   # L 265: eight labels a lane
    (42, 16, 330, 0, 299, 1),   # L 300, HSI
    (43, 12, 430, 0, 399, 0),   # L 400: two 50-vector aggregation slices
    (44, 12, 500, 0, 479, 0),   # L 480
    (45, 10, 700, 0, 640, 0),   # L 641: two cost slices, three scanline vectors a lane
    (46, 8, 1100, 0, 1024, 0),  # L 1025: three cost slices, eight scanline vectors a lane
    (47, 12, 430, 7, 330, 1),   # minD > 0 past 256 labels, HSI
    # the top of the accepted range: L 2048 (four cost slices, eight scanline vectors a
    # lane, the voting decision's 64 KB histogram block) and L 1901 in HSI
    (49, 8, 2100, 0, 2047, 0),
    (50, 6, 1950, 0, 1900, 1),
]


SCAN_STAGES = ("cost_scan", "wta", "outlier", "subpix")
SCAN_CASES = [
    # (seed, H, W, minD, maxD, model, roi, mask)
    (1, 64, 96, 0, 24, 0, False, False),
    (3, 97, 131, 0, 64, 0, False, False),
    (4, 80, 120, 5, 40, 0, False, False),
    (5, 48, 64, 0, 40, 0, False, False),
    (31, 24, 300, 0, 192, 0, False, False),
    (34, 22, 290, 0, 192, 1, False, False),
    (48, 20, 300, 0, 240, 0, False, False),
    (6, 40, 96, 0, 48, 0, True, False),   # ROI / mask: maxD = W/2 (:339-340)
    (7, 40, 96, 0, 48, 1, False, True),
    # very wide rows (the horizontal passes' longest walks, the widest colour-difference rows)
    (52, 5, 4000, 0, 30, 0, False, False),
    (51, 3, 20600, 0, 16, 0, False, False),
]


@pytest.mark.parametrize("case", SCAN_CASES, ids=[f"s{c[0]}_{c[1]}x{c[2]}_d{c[3]}-{c[4]}_m{c[5]}_r{int(c[6])}k{int(c[7])}"
                                             for c in SCAN_CASES])
def test_scanline_and_refine_stages_modes(matcher, tsm, oracle, case):
    """The scanline volumes of both views and the stages after them, in RGB / HSI / ROI /
    mask mode, with and without the racy-schedule emulation, equal the oracle's."""
    seed, H, W, mn, mx, model, roi, mask = case
    left, right = _synthetic(tsm, seed, H, W, mx - mn + 1)
    if roi or mask:  # black out a border band and a block (ROI / mask rules)
        for im in (left, right):
            im[:, :7] = 0
            im[H // 3: H // 2, W // 2: W // 2 + 9] = 0
    for omp in (0, 5):
        d_g, g = _gpu(matcher, tsm, left, right, model, mn, mx, SCAN_STAGES, omp=omp, roi=roi, mask=mask)
        kw = {"scan_emulate_threads": omp} if omp else {}
        d_o, o = oracle.compute(left, right, _oracle_params(oracle, model, mn, mx, roi_matching=int(roi),
                                                           mask_matching=int(mask), **kw), SCAN_STAGES)
        _assert_stages_equal(g, o, SCAN_STAGES)
        assert np.array_equal(d_g, d_o, equal_nan=True)
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    matcher.setOmpEmulation(0)


@pytest.mark.parametrize("case", WIDE, ids=[f"s{c[0]}_{c[1]}x{c[2]}_d{c[3]}-{c[4]}_m{c[5]}" for c in WIDE])
def test_cost_volume_full_label_width(matcher, tsm, oracle, case):
    seed, H, W, mn, mx, model = case
    left, right = _synthetic(tsm, seed, H, W, mx - mn + 1)
    st = ("cost_init", "cost_agg")
    d_g, g = _gpu(matcher, tsm, left, right, model, mn, mx, st)
    d_o, o = oracle.compute(left, right, _oracle_params(oracle, model, mn, mx), st)
    _assert_stages_equal(g, o, st)
    assert np.array_equal(d_g, d_o)


def test_stages_bit_exact_demo_crop(matcher, tsm, oracle, demo_pair_0600):
    l, r = demo_pair_0600
    left, right = l[300:428, 400:656].copy(), r[300:428, 400:656].copy()
    d_g, g = _gpu(matcher, tsm, left, right, 0, 0, 64, STAGES)
    d_o, o = oracle.compute(left, right, _oracle_params(oracle, oracle.RGB, 0, 64), STAGES)
    _assert_stages_equal(g, o, STAGES)
    assert np.array_equal(d_g, d_o)


def test_uniform_image_early_exit(matcher, tsm, oracle):
    # flat images: min_k C(q,k) == 0 leaves scanline pixels untouched (:880-881)
    left = np.full((40, 72, 3), 128, np.uint8)
    right = left.copy()
    d_g, g = _gpu(matcher, tsm, left, right, 0, 0, 16, STAGES)
    d_o, o = oracle.compute(left, right, _oracle_params(oracle, oracle.RGB, 0, 16), STAGES)
    _assert_stages_equal(g, o, STAGES)
    assert np.array_equal(d_g, d_o)


def test_tiny_image_all_border(matcher, tsm, oracle):
    # every census window leaves the image -> cost 2.f everywhere (:562-566)
    rng = np.random.default_rng(7)
    left = rng.integers(0, 256, (6, 8, 3), dtype=np.uint8)
    right = rng.integers(0, 256, (6, 8, 3), dtype=np.uint8)
    d_g, _ = _gpu(matcher, tsm, left, right, 0, 0, 3)
    d_o, _ = oracle.compute(left, right, _oracle_params(oracle, oracle.RGB, 0, 3))
    assert np.array_equal(d_g, d_o)


def test_random_noise_pair(matcher, tsm, oracle):
    # many outliers: exercises the voting carry and interpolation heavily
    rng = np.random.default_rng(11)
    left = rng.integers(0, 256, (70, 110, 3), dtype=np.uint8)
    right = rng.integers(0, 256, (70, 110, 3), dtype=np.uint8)
    d_g, g = _gpu(matcher, tsm, left, right, 0, 0, 30, STAGES)
    d_o, o = oracle.compute(left, right, _oracle_params(oracle, oracle.RGB, 0, 30), STAGES)
    _assert_stages_equal(g, o, STAGES)
    assert np.array_equal(d_g, d_o)


def test_omp_emulation_matches_oracle(matcher, tsm, oracle):
    left, right = _synthetic(tsm, 21, 90, 150, 33)
    for T in (3, 20):
        d_g, g = _gpu(matcher, tsm, left, right, 0, 0, 32, ("cost_scan",), omp=T)
        d_o, o = oracle.compute(left, right, _oracle_params(oracle, oracle.RGB, 0, 32,
                                                           scan_emulate_threads=T), ("cost_scan",))
        _assert_stages_equal(g, o, ("cost_scan",))
        assert np.array_equal(d_g, d_o)


def test_reference_fixture_0600_exact(matcher, tsm, oracle, demo_pair_0600):
    """Full 1280x720, D=[0,192]: with T=20 emulation the GPU output renders to the
    reference's own demo-output/0600_adcensus.png pixel for pixel."""
    left, right = demo_pair_0600
    d_g, _ = _gpu(matcher, tsm, left, right, 0, 0, 192, omp=20)
    ref = load_bgr(os.path.join(GOLDEN, "demo", "0600_adcensus.png"))
    col = oracle.apply_colormap(d_g)
    assert np.array_equal(col, ref), f"{(col != ref).any(-1).sum()} pixels differ"


def test_config_b_serial_bit_exact(matcher, tsm, oracle):
    """The benchmark workload (1242x375, D=[0,192], RGB) at serial semantics."""
    left, right, gt = tsm.synthetic.config_b(1000)
    d_g, _ = _gpu(matcher, tsm, left, right, 0, 0, 192)
    d_o, _ = oracle.compute(left, right, _oracle_params(oracle, oracle.RGB, 0, 192))
    assert np.array_equal(d_g, d_o)
    valid = d_o >= 0
    assert (np.abs(d_g - d_o)[valid] <= 0.5).mean() >= 0.99


def test_batch_equals_single(matcher, tsm):
    pairs = [_synthetic(tsm, 100 + i, 64, 96, 25) for i in range(5)]
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    matcher.setMinMaxDisparity(0, 24)
    matcher.setOmpEmulation(0)
    matcher.setConcurrency(3)
    outs = matcher.compute_batch([p[0] for p in pairs], [p[1] for p in pairs])
    for (l, r), o in zip(pairs, outs):
        assert np.array_equal(o, matcher.compute(l, r))


@pytest.mark.parametrize("mode", ["hsi", "mask", "census7x5", "minD"])
def test_group_equals_single(matcher, tsm, mode):
    """A group of pairs (one pipeline, every launch over the group's pair slots) gives each
    pair exactly its single-pair result, in every model / mode."""
    H, W = 56, 88
    pairs = [_synthetic(tsm, 400 + i, H, W, 33) for i in range(4)]
    if mode == "mask":
        for l, r in pairs:
            l[:, :7] = 0
            r[:, -5:] = 0
    model = tsm.ColorModel.HSI if mode == "hsi" else tsm.ColorModel.RGB
    matcher.setMatchingStrategy(model, False, mode == "mask")
    if mode == "census7x5":
        p = matcher.params()
        p.census_win = 1
        matcher.setParams(p)
    matcher.setMinMaxDisparity(3 if mode == "minD" else 0, 32)
    matcher.setOmpEmulation(0)
    singles = [matcher.compute(l, r) for l, r in pairs]
    for conc in (4, 3):
        matcher.setConcurrency(conc)
        outs = matcher.compute_batch([p[0] for p in pairs], [p[1] for p in pairs])
        for o, s1 in zip(outs, singles):
            assert np.array_equal(o, s1)
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)


def test_api_errors_match_reference(matcher, tsm):
    E = tsm.ADCensusError
    with pytest.raises(E, match=r"^\[ADCensus\] Set MinMaxDisparity error\.$"):
        matcher.setMinMaxDisparity(-5, 5)
    with pytest.raises(E, match=r"^\[ADCensus\] Set MinMaxDisparity error\.$"):
        matcher.setMinMaxDisparity(10, 10)
    with pytest.raises(E, match=r"^\[ADCensus\] Offset must be positive\.$"):
        matcher.setOffset(-1)
    img = np.zeros((16, 16, 3), np.uint8)
    with pytest.raises(E, match=r"^\[ADCensus\] Image error\.$"):
        matcher.compute(img, np.zeros((16, 17, 3), np.uint8))
    with pytest.raises(E, match=r"^\[ADCensus\] Image error\.$"):
        matcher.compute(None, img)
    with pytest.raises(E, match=r"^\[ADCensus\] Image error\.$"):
        matcher.compute(np.zeros((0, 16, 3), np.uint8), np.zeros((0, 16, 3), np.uint8))
    # a failed setter leaves the previous range in place
    matcher.setMinMaxDisparity(0, 32)
    with pytest.raises(E):
        matcher.setMinMaxDisparity(5, 1)
    assert matcher.getMinMaxDisparity() == (0, 32)


def test_default_state_is_reference_default(tsm):
    m = tsm.ADCensus(0)
    assert m.getMinMaxDisparity() == (0, 64)  # ADCensus.cpp:411-412
    p = m.params()
    assert (p.color_thresh1, p.max_length1, p.color_diff) == (5, 17, 3)  # HSI set (:413-414)
    m.close()


def test_hsi_mode_against_oracle(matcher, tsm, oracle):
    """HSI ("Selective AD-Census-HSI", the reference's default model), every stage
    bit-exact: bgr2hsi's hue byte (acosf, :1456) comes from the host-built conversion table,
    so the converted images equal the oracle's byte for byte."""
    left, right = _synthetic(tsm, 31, 72, 120, 33)
    d_g, g = _gpu(matcher, tsm, left, right, 1, 0, 32, STAGES)
    d_o, o = oracle.compute(left, right, _oracle_params(oracle, oracle.HSI, 0, 32), STAGES)
    _assert_stages_equal(g, o, STAGES)
    assert np.array_equal(d_g, d_o)


def test_hsi_conversion_every_colour(matcher, tsm, oracle):
    """bgr2hsi over all 2^24 BGR colours (a 4096 x 4096 image, each colour once), with and
    without the mask-mode hue filter: the device table equals the oracle's conversion."""
    c = np.arange(1 << 24, dtype=np.uint32)
    img = np.stack([c & 0xff, (c >> 8) & 0xff, c >> 16], -1).astype(np.uint8).reshape(4096, 4096, 3)
    for mask in (False, True):
        matcher.setMatchingStrategy(tsm.ColorModel.HSI, False, mask)
        got = matcher.convert_hsi(img)
        exp = oracle.bgr2hsi(img, filter=int(mask))
        if not np.array_equal(got, exp):
            bad = np.argwhere((got != exp).any(-1))
            pytest.fail(f"mask={mask}: {len(bad)} colours differ, first BGR {tuple(img[tuple(bad[0])])}: "
                        f"gpu={tuple(got[tuple(bad[0])])} oracle={tuple(exp[tuple(bad[0])])}")
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)


@pytest.mark.parametrize("roi,mask,model,W", [(True, False, 0, 100), (False, True, 0, 100),
                                              (True, False, 1, 100), (False, True, 1, 100),
                                              (False, True, 0, 600), (True, False, 1, 560),
                                              (True, False, 0, 1300)],
                         ids=["roi", "mask", "roi_hsi", "mask_hsi", "mask_L301", "roi_hsi_L281", "roi_L651"])
def test_roi_mask_modes(matcher, tsm, oracle, roi, mask, model, W):
    """ROI / mask matching: maxD := W/2 (:339-340), black pixels excluded from costs,
    arms and scanline (:459-460, :551-555, :625-629, :824, :862), offset and background
    rules on the output (:388-403, :1415-1427)."""
    Hh = 64 if W <= 100 else 12
    left, right = _synthetic(tsm, 41, Hh, W, min(W // 2 + 1, 120))
    left[:, :12] = 0    # black (masked) band
    right[:, -9:] = 0
    matcher.setOffset(3)
    d_g, _ = _gpu(matcher, tsm, left, right, model, 0, 50, roi=roi, mask=mask)
    matcher.setOffset(0)
    p = _oracle_params(oracle, model, 0, 50, roi_matching=int(roi), mask_matching=int(mask),
                       offset=3)
    d_o, _ = oracle.compute(left, right, p)
    assert np.array_equal(d_g, d_o)
    assert matcher.getMinMaxDisparity() == (0, W // 2)  # maxD = W/2 persists (:340)
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)


def test_census_7x5_window(matcher, tsm, oracle):
    """CensusWin::CENSUSWIN_7x5 (stereo_utils.h:203) through tsm_adc_set_params."""
    left, right = _synthetic(tsm, 51, 64, 96, 25)
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    p = matcher.params()
    p.census_win = 1
    matcher.setParams(p)
    matcher.setMinMaxDisparity(0, 24)
    matcher.setOmpEmulation(0)
    d_g, g = matcher.compute_debug(left, right, STAGES)
    d_o, o = oracle.compute(left, right, _oracle_params(oracle, oracle.RGB, 0, 24, census_win=1), STAGES)
    _assert_stages_equal(g, o, STAGES)
    assert np.array_equal(d_g, d_o)
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)  # resets the parameter set
    assert matcher.params().census_win == 0


@pytest.mark.parametrize("cfg", ["C", "E", "BIG49"])
def test_full_size_configs_bit_exact(matcher, tsm, cfg):
    """Configs C (1500x1000, D=[0,256]) and E (2048x1536 grey, D=[0,320]) at full size, and
    a 2400x1600 D=[0,192] pair (a 6 GB volume: the 64-bit aggregation path at 49 label
    vectors): the SHA-256 of the final fp32 disparity equals the oracle's, recorded by
    tests/golden/make_config_hashes.py (its oracle runs take minutes)."""
    import hashlib
    import json

    gold = json.load(open(os.path.join(GOLDEN, "config_hashes.json")))[cfg]
    gen = {"C": tsm.synthetic.config_c, "E": tsm.synthetic.config_e,
           "BIG49": lambda: tsm.synthetic.make_scene(4000, 1600, 2400, 193)}[cfg]
    left, right, _ = gen()
    d_g, _ = _gpu(matcher, tsm, left, right, 0, 0, gold["max_disparity"])
    d_g = np.ascontiguousarray(d_g, dtype=np.float32)
    assert list(d_g.shape) == gold["shape"]
    assert abs(float((d_g >= 0).mean()) - gold["valid_fraction"]) < 1e-12
    assert hashlib.sha256(d_g.tobytes()).hexdigest() == gold["sha256"]


@pytest.mark.parametrize("key,model,omp", [("B_HSI_1000", 1, 0), ("B_OMP20_1000", 0, 20)])
def test_config_b_modes_full_size(matcher, tsm, key, model, omp):
    """Config B pair 1000 in the reference's default HSI model, and in RGB with the T = 20
    race emulation (the mode equal to the reference's shipped outputs): SHA-256 of the fp32
    disparity == the oracle's (the bench's configs block checks the same hashes)."""
    import hashlib
    import json

    gold = json.load(open(os.path.join(GOLDEN, "config_hashes.json")))[key]
    left, right, _ = tsm.synthetic.config_b(1000)
    try:
        d_g, _ = _gpu(matcher, tsm, left, right, model, 0, 192, omp=omp)
    finally:  # the shared matcher goes back to the serial RGB mode even on failure
        matcher.setOmpEmulation(0)
        matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    d_g = np.ascontiguousarray(d_g, dtype=np.float32)
    assert hashlib.sha256(d_g.tobytes()).hexdigest() == gold["sha256"]


PARAM_CASES = [
    # tsm_adc_set_params beyond the defaults (ADCensusParams, stereo_utils.h:209-244):
    # every field the kernels read, against the oracle, bit-exact
    ("arms8", 0, dict(max_length1=8, max_length2=4)),
    ("arms41", 0, dict(max_length1=41, max_length2=20, color_thresh1=40)),   # the streamers' longest arm
    ("arms60", 0, dict(max_length1=60, max_length2=30, color_thresh1=40)),   # one-pass-a-launch path
    ("arms128", 1, dict(max_length1=128, max_length2=64, intensity_thresh1=60)),
    ("iter2", 0, dict(iterations=2)),
    ("iter6", 1, dict(iterations=6)),
    ("iter0", 0, dict(iterations=0)),
    ("p1p2", 0, dict(pi1=0.5, pi2=5.0, color_diff=25)),
    ("voting", 0, dict(voting_thresh=8, voting_ratio_thresh=0.6, disp_tolerance=1, max_search_depth=7)),
    ("canny", 1, dict(canny_thresh1=60, canny_thresh2=15, color_thresh2=3)),
    ("lambdas", 0, dict(lambda_ad=7.5, lambda_census=21.0, census_win=1)),
]


@pytest.mark.parametrize("name,model,kw", PARAM_CASES, ids=[c[0] for c in PARAM_CASES])
def test_params_matrix(matcher, tsm, oracle, name, model, kw):
    left, right = _synthetic(tsm, 60, 70, 120, 33)
    matcher.setMatchingStrategy(tsm.ColorModel(model))
    p = matcher.params()
    for k, v in kw.items():
        setattr(p, k, v)
    matcher.setParams(p)
    matcher.setMinMaxDisparity(0, 32)
    matcher.setOmpEmulation(0)
    d_g, g = matcher.compute_debug(left, right, STAGES)
    d_o, o = oracle.compute(left, right, _oracle_params(oracle, model, 0, 32, **kw), STAGES)
    _assert_stages_equal(g, o, STAGES)
    assert np.array_equal(d_g, d_o)
    matcher.setMatchingStrategy(tsm.ColorModel.RGB)  # resets the parameter set


def test_params_refused(matcher, tsm):
    """What the kernels cannot do exactly is refused, not approximated."""
    base = matcher.params()
    for k, v in (("blur_kernel_size", 5), ("canny_kernel_size", 5), ("voting_thresh", 21),
                 ("max_length1", 257), ("max_length1", 0), ("census_win", 2), ("color_diff", 255),
                 ("iterations", -1)):
        p = matcher.params()
        setattr(p, k, v)
        with pytest.raises((RuntimeError, tsm.ADCensusError)):
            matcher.setParams(p)
        assert getattr(matcher.params(), k) == getattr(base, k)


def test_reference_fixture_0045_exact(matcher, tsm, oracle, demo_pair_0045):
    """Full 1280x720, D=[0,192]: the GPU output at T=20 renders to the reference's own
    demo-output/0045_ADCensus.png pixel for pixel."""
    left, right = demo_pair_0045
    d_g, _ = _gpu(matcher, tsm, left, right, 0, 0, 192, omp=20)
    ref = load_bgr(os.path.join(GOLDEN, "demo", "0045_ADCensus.png"))
    col = oracle.apply_colormap(d_g)
    assert np.array_equal(col, ref), f"{(col != ref).any(-1).sum()} pixels differ"


@pytest.mark.parametrize("case", ["MOTO", "ROI_0600", "MASK_HSI_0600", "A_0600", "A_0600_OMP20"])
def test_real_pairs_full_size(matcher, tsm, demo_pair_0600, case):
    """The reference's real demo pairs at full size against oracle hashes
    (tests/golden/make_config_hashes.py): the Middlebury Motorcycle pair of config C
    (1482x994, D=[0,256]); 0600 (1280x720) in ROI mode (maxD := W/2 = 640, 641 labels) and in
    mask mode with the reference's default HSI model; 0600 at D=[0,192] serial and with the
    T = 20 race emulation (BASELINE configs[0], the bench's A_real entries)."""
    import hashlib
    import json

    gold = json.load(open(os.path.join(GOLDEN, "config_hashes.json"))).get(case)
    if gold is None:
        pytest.fail(f"no committed oracle hash for {case}")
    if case == "MOTO":
        d = os.path.join(GOLDEN, "demo")
        left, right = load_bgr(os.path.join(d, "Motorcycle_Left.png")), load_bgr(os.path.join(d, "Motorcycle_Right.png"))
    else:
        left, right = demo_pair_0600
    model = gold.get("color_model", 0)
    try:
        d_g, _ = _gpu(matcher, tsm, left, right, model, 0, gold["max_disparity"],
                      roi=bool(gold.get("roi_matching", 0)), mask=bool(gold.get("mask_matching", 0)),
                      omp=gold.get("scan_emulate_threads", 0))
    finally:
        matcher.setOmpEmulation(0)
        matcher.setMatchingStrategy(tsm.ColorModel.RGB)
    d_g = np.ascontiguousarray(d_g, dtype=np.float32)
    assert list(d_g.shape) == gold["shape"]
    assert abs(float((d_g >= 0).mean()) - gold["valid_fraction"]) < 1e-12
    assert hashlib.sha256(d_g.tobytes()).hexdigest() == gold["sha256"]


@pytest.mark.parametrize("seed", [1000, 1127])
def test_config_b_noisy_full_size(matcher, tsm, seed):
    """Config B with independent +-3 noise on the right view (synthetic.config_b_noisy, the
    bench's B_noisy entry): no exact-zero aggregated minima, so the scanline updates and
    stores every vector.  SHA-256 of the fp32 disparity == the oracle's."""
    import hashlib
    import json

    gold = json.load(open(os.path.join(GOLDEN, "config_hashes.json")))[f"B_NOISY_{seed}"]
    left, right, _ = tsm.synthetic.config_b_noisy(seed)
    d_g, _ = _gpu(matcher, tsm, left, right, 0, 0, 192)
    d_g = np.ascontiguousarray(d_g, dtype=np.float32)
    assert hashlib.sha256(d_g.tobytes()).hexdigest() == gold["sha256"]
