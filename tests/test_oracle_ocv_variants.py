"""Known-answer tests of the oracle's OpenCV build-variant switches ("OpenCV
semantics targets"). The reference pins OpenCV only by ROS distro (melodic -> 3.2.0,
noetic -> 4.2.0; .github/workflows/ros-build.yml:14-21, CMakeLists.txt:48-51) and OpenCV is
absent here, so each divergence between versions / between computeDisparitySGBM's scalar
and CV_SIMD branches is a switch of the restatement. Each test shows that the two
behaviours differ on a constructed input and where they agree. The bits come from
`sgm_params.ocv_compat` (default COMPAT_MELODIC, the reference's Dockerfile build) OR-ed with the
process-wide switch these KATs use; the GPU engine reproduces every combination bit-exactly
(tests/test_gpu_ocv_compat.py).
"""
import numpy as np
import pytest

from conftest import to_oracle_params  # noqa: F401  (fixture module)


def _pair(synth, h, w, minD, D, seed):
    left, right, _ = synth.stereo_pair(h, w, minD, D, seed=seed)
    return left, right


def _ocv(oracle, mode, **kw):
    m = oracle.MODE_OCV_SGBM5 if mode == "sgbm" else oracle.MODE_OCV_HH8
    base = dict(min_disparity=0, num_disparities=32, block_size=5, p1=8, p2=64, uniqueness_ratio=10,
                prefilter_cap=31, speckle_window_size=0, speckle_range=0, ocv_compat=0)
    base.update(kw)
    return oracle.make_params(m, **base)


@pytest.mark.parametrize("mode", ["sgbm", "hh"])
def test_col0_legacy_cost_volume(oracle, synth, mode):
    """3.x's vertical update loop starts at column 1: C' column 0 (x = minX1) keeps its row-0
    value (MODE_SGBM, one running C row) or the P2 initialisation (MODE_HH), every other
    column is unchanged."""
    left, right = _pair(synth, 40, 96, 0, 32, seed=3)
    p = _ocv(oracle, mode)
    ref = oracle.ocv_cost(p, left, right)
    with oracle.ocv_compat(oracle.OCV_COL0_LEGACY):
        leg = oracle.ocv_cost(p, left, right)
    assert np.array_equal(leg[:, 1:], ref[:, 1:])
    assert np.array_equal(leg[0, 0], ref[0, 0])
    if mode == "sgbm":
        assert (leg[1:, 0] == leg[0, 0]).all()
    else:
        assert (leg[1:, 0] == p.p2).all()
    assert not np.array_equal(leg[1:, 0], ref[1:, 0])
    # the disparity maps differ (column 0 seeds the left-to-right paths of every row)
    d_ref = oracle.match(p, left, right)
    with oracle.ocv_compat(oracle.OCV_COL0_LEGACY):
        d_leg = oracle.match(p, left, right)
    assert not np.array_equal(d_ref, d_leg)


@pytest.mark.parametrize("mode", ["sgbm", "hh"])
def test_simd_saturation_agrees_without_overflow(oracle, synth, mode):
    """The CV_SIMD branch saturates int16 where the scalar one wraps / sums in int; with the
    node defaults (block 15, cap 31: box bound 225 * 125 + 400 = 28525 < 32767) no value
    leaves int16 and the two agree bit for bit."""
    left, right = _pair(synth, 64, 160, 9, 64, seed=5)
    p = _ocv(oracle, mode, min_disparity=9, num_disparities=64, block_size=15, p1=200, p2=400,
             uniqueness_ratio=15, prefilter_cap=31, speckle_window_size=100, speckle_range=4)
    ref = oracle.match(p, left, right)
    with oracle.ocv_compat(oracle.OCV_SIMD_SAT):
        simd = oracle.match(p, left, right)
    assert np.array_equal(ref, simd)


@pytest.mark.parametrize("mode", ["sgbm", "hh"])
def test_simd_saturation_differs_on_overflow(oracle, mode):
    """Block 21 at preFilterCap 63 on binary (0/255) noise against its negative: box sums pass 32767,
    the scalar C' wraps while the SIMD running sums of rows y > 0 clip at 32767, so cost volumes
    and disparities differ."""
    rng = np.random.default_rng(1)
    left = (rng.integers(0, 2, (64, 160)) * 255).astype(np.uint8)
    right = 255 - left                          # every match maximally dissimilar
    p = _ocv(oracle, mode, block_size=21, prefilter_cap=63, p1=50, p2=3000, uniqueness_ratio=0)
    c_ref = oracle.ocv_cost(p, left, right)
    with oracle.ocv_compat(oracle.OCV_SIMD_SAT):
        c_simd = oracle.ocv_cost(p, left, right)
        d_simd = oracle.match(p, left, right)
    assert (c_ref < 0).any(), "the scalar cost volume should wrap on this input"
    # (row 0's accumulation is the scalar loop in every build, so it may wrap in both)
    assert (c_simd == 32767).any() and not np.array_equal(c_ref, c_simd)
    assert not np.array_equal(oracle.match(p, left, right), d_simd)


def _tie_volume(D, ties, h=1, w1=1, base=500, low=100):
    S = np.full((h, w1, D), base, np.uint16)
    for d in ties:
        S[..., d] = low
    return S


def test_lane_tie_rule_on_constructed_sums(oracle):
    """MODE_SGBM's SSE2 WTA keeps a strict minimum per 8-lane slot and takes the lowest lane
    holding the overall minimum: equal minima at d = 7 (lane 7) and d = 16 (lane 0) give 16,
    where the scalar loop (and MODE_HH in either build) gives 7. A tie inside one lane
    (d = 3, 11) gives the smaller d in both."""
    D, minD = 32, 0
    w = D + 1                       # width1 = 1: one pixel per row
    p5 = _ocv(oracle, "sgbm", num_disparities=D, min_disparity=minD, uniqueness_ratio=0)
    p8 = _ocv(oracle, "hh", num_disparities=D, min_disparity=minD, uniqueness_ratio=0)
    S = _tie_volume(D, (7, 16))
    S2 = _tie_volume(D, (3, 11))
    assert oracle.wta(p5, S, w)[0, D] == 7 * 16
    with oracle.ocv_compat(oracle.OCV_LANE_TIE):
        assert oracle.wta(p5, S, w)[0, D] == 16 * 16
        assert oracle.wta(p8, S, w)[0, D] == 7 * 16      # MODE_HH's WTA is the scalar loop
        assert oracle.wta(p5, S2, w)[0, D] == 3 * 16
    assert oracle.wta(p5, S2, w)[0, D] == 3 * 16


def test_lane_tie_rule_changes_a_match(oracle):
    """A 9-periodic texture makes S(d) and S(d + 9) tie across lanes; the lane rule moves some
    winners (and only MODE_SGBM's)."""
    rng = np.random.default_rng(4)
    tile = rng.integers(0, 256, (64, 9), dtype=np.uint8)
    img = np.tile(tile, (1, 24))[:, :200].copy()
    right = np.roll(img, -7, axis=1)            # true disparity 7 ~ 16 ~ 25: lanes 7, 0, 1
    p5 = _ocv(oracle, "sgbm", num_disparities=32, uniqueness_ratio=0, block_size=3)
    p8 = _ocv(oracle, "hh", num_disparities=32, uniqueness_ratio=0, block_size=3)
    d5, d8 = oracle.match(p5, img, right), oracle.match(p8, img, right)
    with oracle.ocv_compat(oracle.OCV_LANE_TIE):
        l5, l8 = oracle.match(p5, img, right), oracle.match(p8, img, right)
    assert np.array_equal(d8, l8)
    assert not np.array_equal(d5, l5)


def test_default_is_the_engine_restatement(oracle, synth):
    """The process-wide switch is off by default (the parameter block decides) and restored by
    the context manager; the parameter default is the melodic build."""
    assert oracle.make_params(oracle.MODE_OCV_SGBM5).ocv_compat == oracle.COMPAT_MELODIC == 7
    assert oracle.make_params(oracle.MODE_CENSUS8).ocv_compat == 0
    assert oracle.lib().sgmref_get_ocv_compat() == 0
    with oracle.ocv_compat(7):
        assert oracle.lib().sgmref_get_ocv_compat() == 7
    assert oracle.lib().sgmref_get_ocv_compat() == 0
