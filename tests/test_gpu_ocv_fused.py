"""GPU parity of the fused OpenCV cost kernel (`k_ocv_cost_fused`, csrc/ocv_sgm.hip) with it forced.

The fused kernel (Birchfield-Tomasi pixel cost + vertical box + horizontal box + P2 in one pass)
is the default on every frame of >= 10^8 cells, i.e. every production-size frame: the shipped
2448x2048 D=480 block-21 configuration (/root/reference/launch/stereo_matcher.launch:36-46) and
1080p. Small frames take the two-kernel form by default, so here `SGM_OCV_FUSED=1` forces the
fused kernel on small frames and `SGM_FUSE_DPC` forces each disparity-pair block width (8, 16,
32 pairs; a width the geometry cannot take falls back as the launcher does), `SGM_FUSE_ROWS`
forces short bands (many band seams, each with its 2*SH2 warm-up rows). Every case is compared
bit for bit with the oracle's C' (oracle/sgm_oracle.c) and, for a subset,
the whole match; `SGM_OCV_FUSED=0` runs the same cases through the unfused kernels.
Covered: every odd block 1-21, D % 32 != 0 (the 8-pair blocks), D % 64 == 0, negative minD,
frames narrower than one strip, heights below one band and below the box, the column-0 rule
(COL0_LEGACY), SIMD_SAT frames whose overflow flag routes them to the saturating cost (wide == 2).
"""
import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu


def fusable(h, w, minD, D, block, cap):
    """ocv_cost_fusable() of csrc/ocv_sgm.hip without the size default (the kernel is forced)."""
    ftzero = max(cap, 15) | 1
    sh2 = block // 2
    width1 = (w + min(minD, 0)) - max(minD + D, 0)
    return sh2 <= 10 and (block * block) * (2 * ftzero + 63) <= 65535 and 2 * ftzero + 63 <= 255 and width1 > 0


# (h, w, minD, D, block, cap, compat): compat cycles over scalar / column-0 rule / melodic
GEOMS = [
    (12, 50, 0, 16, 5, 31, 0),          # H below one band
    (9, 45, 4, 16, 7, 15, 1),
    (4, 40, -3, 16, 9, 63, 7),          # H below the box
    (17, 70, 2, 32, 3, 1, 0),
    (40, 200, 9, 64, 15, 31, 1),
    (30, 300, 0, 128, 11, 20, 7),
    (130, 333, 5, 48, 9, 31, 0),        # D % 32 = 16: 16-pair blocks have a half-empty last chunk
    (70, 400, -8, 80, 21, 7, 7),        # block 21 with D % 32 = 16
    (150, 500, 0, 96, 1, 31, 1),        # block 1
    (64, 150, 10, 128, 5, 31, 7),       # width1 = 12: one narrow strip, both frame edges in it
    (50, 700, -5, 144, 13, 15, 0),
    (90, 460, 3, 192, 17, 15, 1),
    (33, 900, 147, 480, 21, 7, 7),      # the shipped geometry's D, minD and box
    (26, 1200, 0, 256, 19, 11, 0),      # width1 > 7 strips
    (24, 1000, 0, 752, 21, 7, 7),       # the processing launch's D = 752: 16-pair blocks, partial last chunk
    (40, 620, 3, 272, 5, 31, 0),        # D % 32 = 16 above 256 (16 pairs by default)
]


@pytest.mark.parametrize("rows", ["", "16"], ids=["bands-auto", "bands-16"])
@pytest.mark.parametrize("dpc", ["8", "16", "32"])
@pytest.mark.parametrize("geom", GEOMS, ids=[f"{g[0]}x{g[1]}-m{g[2]}-D{g[3]}-b{g[4]}-c{g[6]}" for g in GEOMS])
def test_fused_cost_volume(engine, oracle, pkg, monkeypatch, geom, dpc, rows):
    h, w, minD, D, block, cap, compat = geom
    assert fusable(h, w, minD, D, block, cap)
    monkeypatch.setenv("SGM_OCV_FUSED", "1")
    monkeypatch.setenv("SGM_FUSE_DPC", dpc)
    if rows:
        monkeypatch.setenv("SGM_FUSE_ROWS", rows)
    rng = np.random.default_rng(h * w + D + block)
    left = rng.integers(0, 256, (h, w), dtype=np.uint8)
    right = rng.integers(0, 256, (h, w), dtype=np.uint8)
    p = pkg.default_params(0, min_disparity=minD, num_disparities=D, block_size=block, prefilter_cap=cap,
                           p1=8, p2=32, ocv_compat=compat)
    engine.set_params(p)
    got = engine.ocv_cost(left, right)
    ref = oracle.ocv_cost(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} cost cells differ"


@pytest.mark.parametrize("fused", ["0", "1"])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("geom", GEOMS[::2], ids=[f"{g[0]}x{g[1]}-D{g[3]}-b{g[4]}" for g in GEOMS[::2]])
def test_fused_match(engine, oracle, synth, pkg, monkeypatch, geom, mode, fused):
    """The whole match (paths, WTA, median, speckles) over the fused and the unfused cost."""
    h, w, minD, D, block, cap, compat = geom
    monkeypatch.setenv("SGM_OCV_FUSED", fused)
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=h + w + D)
    p = pkg.default_params(mode, min_disparity=minD, num_disparities=D, block_size=block, prefilter_cap=cap,
                           ocv_compat=compat)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("compat", [7, 2, 0], ids=["melodic", "noetic", "scalar"])
@pytest.mark.parametrize("dpc", ["8", "16"])
def test_fused_cost_overflow_flag(engine, oracle, pkg, monkeypatch, compat, dpc):
    """Binary 0/255 frames at block 15, cap 40, P2 chosen so the largest box sum + P2 passes 32767: the fused
    kernel's overflow flag (max box sum > ovf_thr - P2) routes the SIMD builds to their
    saturating cost (wide == 2) and the scalar build to int32 volumes; C' and the match bit-exact."""
    monkeypatch.setenv("SGM_OCV_FUSED", "1")
    monkeypatch.setenv("SGM_FUSE_DPC", dpc)
    rng = np.random.default_rng(3)
    left = (rng.integers(0, 2, (48, 400)) * 255).astype(np.uint8)
    right = np.where(rng.random((48, 400)) < 0.8, 255 - left, left).astype(np.uint8)
    kw = dict(min_disparity=0, num_disparities=64, block_size=15, prefilter_cap=40, p1=30, speckle_window_size=0)
    assert fusable(48, 400, 0, 64, 15, 40)
    box_max = int(oracle.ocv_cost(oracle.make_params(0, p2=100, ocv_compat=0, **kw), left, right).max()) - 100
    p2 = 32767 + 100 - box_max                                 # the largest C' passes 32767 by 100
    p = pkg.default_params(0, ocv_compat=compat, p2=p2, **kw)
    engine.set_params(p)
    op = to_oracle_params(oracle, p)
    ref = oracle.ocv_cost(op, left, right)
    assert int(ref.max()) > 32767 - p2 or (ref < 0).any()      # the frame is in the overflow regime
    got = engine.ocv_cost(left, right)
    assert np.array_equal(got, ref), f"C': {(got != ref).sum()} cells differ"
    m = engine.match(left, right)
    mref = oracle.match(op, left, right)
    assert np.array_equal(m, mref), f"match: {(m != mref).sum()} pixels differ"


@pytest.mark.parametrize("compat", [7, 0], ids=["melodic", "scalar"])
def test_fused_cost_1080p_all_pair_widths(engine, oracle, synth, pkg, monkeypatch, compat):
    """1920x1080 D=128 block 5 (fused by default) with each disparity-pair block width forced:
    the full-size band and strip layout of every instantiation against the oracle's C'."""
    left, right, _ = synth.stereo_pair(1080, 1920, 0, 128, seed=1081)
    p = pkg.default_params(0, min_disparity=0, num_disparities=128, block_size=5, ocv_compat=compat)
    engine.set_params(p)
    ref = oracle.ocv_cost(to_oracle_params(oracle, p), left, right)
    for dpc in ("8", "16", "32"):
        monkeypatch.setenv("SGM_FUSE_DPC", dpc)
        got = engine.ocv_cost(left, right)
        assert np.array_equal(got, ref), f"DPC {dpc}: {(got != ref).sum()} cells differ"
        del got
