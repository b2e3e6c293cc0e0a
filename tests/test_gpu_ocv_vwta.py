"""GPU parity — the OpenCV modes with the vertical direction of the last group fused into the
WTA (ocv_sgm.hip k_ocv_vwta + the rowfin epilogue, forced by SGM_OCV_VWTA=1): MODE_SGBM's ↓
and MODE_HH's ↑ are never stored, their costs enter S in OpenCV's saturating order from
registers. Bit-exact against the CPU restatement in every build variant (ocv_compat), both
volume regimes (int16, and the flagged int32 / saturating kernels) and every line shape
(DPL 1-32 per 64-lane line, D up to 2048)."""
import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu

GEOMS = [(0, 480, 640, 9, 64, 15, 0), (1, 96, 500, 0, 128, 5, 0), (0, 40, 600, -4, 256, 7, 50),
         (1, 33, 200, 3, 48, 3, 0), (1, 24, 640, -3, 480, 9, 0), (0, 20, 700, 147, 400, 21, 100),
         (0, 31, 170, 0, 16, 5, 0), (1, 18, 1400, -7, 784, 3, 0), (0, 14, 1300, 0, 1024, 5, 0),
         (0, 12, 2200, 5, 2048, 3, 0), (1, 3, 90, 0, 32, 5, 0)]


@pytest.mark.parametrize("compat", [0, 2, 7], ids=["scalar", "noetic", "melodic"])
@pytest.mark.parametrize("mode,h,w,minD,D,block,spk", GEOMS, ids=[str(i) for i in range(len(GEOMS))])
def test_ocv_vwta_pipeline(engine, oracle, synth, pkg, monkeypatch, compat, mode, h, w, minD, D, block, spk):
    monkeypatch.setenv("SGM_OCV_VWTA", "1")
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=h * 7 + D)
    p = pkg.default_params(mode, min_disparity=minD, num_disparities=D, block_size=block, ocv_compat=compat,
                           speckle_window_size=spk)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("compat", [0, 7], ids=["scalar", "melodic"])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("force", ["", "1"], ids=["auto", "forced"])
def test_ocv_vwta_wide_path_costs(engine, oracle, synth, pkg, monkeypatch, mode, force, compat):
    """The overflow regime (int32 volumes, or the SIMD build's saturating kernels) through the
    fused kernel: wrapped boxes (21x21, preFilterCap 62), and an ordinary frame forced through
    the flagged kernels (SGM_OCV_WIDE=1)."""
    monkeypatch.setenv("SGM_OCV_VWTA", "1")
    if force:
        monkeypatch.setenv("SGM_OCV_WIDE", force)
        kw = dict(min_disparity=-4, num_disparities=48, block_size=5)
        left, right, _ = synth.stereo_pair(37, 160, 0, 48, seed=5)
    else:
        kw = dict(min_disparity=-4, num_disparities=48, block_size=21, p1=106, p2=834, prefilter_cap=62,
                  uniqueness_ratio=99, disp12_max_diff=5)
        rng = np.random.default_rng(871)
        left = np.full((9, 118), 90, dtype=np.uint8)
        left[:, ::3] = rng.integers(0, 256, (9, 40), dtype=np.uint8)
        right = np.roll(left, -3, axis=1)
    p = pkg.default_params(mode, speckle_window_size=0, ocv_compat=compat, **kw)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("uniq", [0, 10])
def test_ocv_vwta_saturated_sums(engine, oracle, pkg, monkeypatch, mode, uniq):
    """Pixels whose S saturates at MAX_COST for every d stay INVALID (bestDisp = -1)."""
    monkeypatch.setenv("SGM_OCV_VWTA", "1")
    rng = np.random.default_rng(56 + mode)
    left = rng.integers(0, 256, (24, 200), dtype=np.uint8)
    right = rng.integers(0, 256, (24, 200), dtype=np.uint8)
    p = pkg.default_params(mode, min_disparity=-3, num_disparities=128, block_size=21, p1=128, p2=912,
                           uniqueness_ratio=uniq, prefilter_cap=27, speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("mode", [0, 1])
def test_ocv_vwta_equals_unfused_on_the_shipped_config_crop(engine, synth, pkg, monkeypatch, mode):
    """The reference's shipped launch configuration (2448 wide, minD 147, D 480, block 21,
    cap 7, P1 200 / P2 400, uniqueness 2, speckle 1000/4) on a 2448 x 160 crop: the fused
    kernel and paths + WTA agree bit for bit (the full frame takes the fused kernel by
    default, test_gpu_refcfg.py)."""
    left, right, _ = synth.stereo_pair(160, 2448, 147, 480, seed=2448)
    p = pkg.default_params(mode, min_disparity=147, num_disparities=480, block_size=21, uniqueness_ratio=2,
                           speckle_window_size=1000, speckle_range=4, prefilter_cap=7, p1=200, p2=400)
    engine.set_params(p)
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("SGM_OCV_VWTA", v)
        outs.append(engine.match(left, right))
    assert np.array_equal(outs[0], outs[1]), f"{(outs[0] != outs[1]).sum()} pixels differ"
