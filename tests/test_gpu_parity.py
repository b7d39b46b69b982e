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
]


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
    """HSI ("Selective AD-Census-HSI", the reference's default model).  bgr2hsi uses
    acosf (device libm vs glibc): the converted images may differ in rare hue bytes, so
    the images are compared with a tolerance and the disparity on >= 99 % of pixels."""
    left, right = _synthetic(tsm, 31, 72, 120, 33)
    d_g, g = _gpu(matcher, tsm, left, right, 1, 0, 32, ("images",))
    d_o, o = oracle.compute(left, right, _oracle_params(oracle, oracle.HSI, 0, 32), ("images",))
    img_diff = np.abs(g["images"].astype(int) - o["images"].astype(int))
    assert (img_diff <= 1).all()
    assert (img_diff > 0).mean() < 1e-3
    if (img_diff == 0).all():
        assert np.array_equal(d_g, d_o)
    valid = d_o >= 0
    assert (np.abs(d_g - d_o)[valid] <= 0.5).mean() >= 0.99


@pytest.mark.parametrize("roi,mask", [(True, False), (False, True)])
def test_roi_mask_modes(matcher, tsm, oracle, roi, mask):
    """ROI / mask matching: maxD := W/2 (:339-340), black pixels excluded from costs,
    arms and scanline (:459-460, :551-555, :625-629, :824, :862), offset and background
    rules on the output (:388-403, :1415-1427)."""
    left, right = _synthetic(tsm, 41, 64, 100, 51)
    left[:, :12] = 0    # black (masked) band
    right[:, -9:] = 0
    matcher.setOffset(3)
    d_g, _ = _gpu(matcher, tsm, left, right, 0, 0, 50, roi=roi, mask=mask)
    matcher.setOffset(0)
    p = _oracle_params(oracle, oracle.RGB, 0, 50, roi_matching=int(roi), mask_matching=int(mask),
                       offset=3)
    d_o, _ = oracle.compute(left, right, p)
    assert np.array_equal(d_g, d_o)
    assert matcher.getMinMaxDisparity() == (0, 50)  # maxD = W/2 persists (:340)


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


MFMA_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import tea_stereo_matching_amd as T
out = sys.argv[2]
res = {}
m = T.ADCensus(0)
for i, (seed, H, W, mn, mx) in enumerate(((31, 24, 300, 0, 192), (2, 120, 160, 0, 48), (3, 97, 131, 0, 64))):
    left, right = T.synthetic.make_scene(seed, H, W, mx - mn + 1)[:2]
    m.setMatchingStrategy(T.ColorModel(0), False, False)
    m.setMinMaxDisparity(mn, mx)
    _, g = m.compute_debug(left, right, ("cost_init",))
    res[f"c{i}"] = g["cost_init"]
m.close()
np.savez(out, **res)
"""


def test_cost_mfma_experiment_bit_exact(oracle, tmp_path):
    """The opt-in matrix-core cost build (TSM_COST_MFMA=1, an experiment kept beside the
    popcount walk) produces the oracle's initial volume bit for bit.  The switch is read
    once per process, so the build runs in a child process."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / "mfma.npz")
    env = dict(os.environ, TSM_COST_MFMA="1")
    r = subprocess.run([sys.executable, "-c", MFMA_CHILD, root, out], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.load(out)
    for i, (seed, H, W, mn, mx) in enumerate(((31, 24, 300, 0, 192), (2, 120, 160, 0, 48), (3, 97, 131, 0, 64))):
        left, right = _synthetic(__import__("tea_stereo_matching_amd"), seed, H, W, mx - mn + 1)
        _, o = oracle.compute(left, right, _oracle_params(oracle, oracle.RGB, mn, mx), ("cost_init",))
        assert np.array_equal(got[f"c{i}"], o["cost_init"]), f"case {i}"
