"""GPU parity of the OpenCV modes with the path volumes as deficit records / planes (Geom::evol).

In the plain int16 regime every path cost is L = C' - e with e in [0, P2] (OpenCV's recurrence,
SURVEY Appendix A.5), so for P2 <= 511 the path kernel stores e in 9 bits instead of L in 16 and
the WTA kernels rebuild L from C' (csrc/ocv_sgm.hip `load_e`, `evol_store`, `ocv_evol_mode`). The
layout is picked by D (records per pixel, or byte + bit planes when D % 128 == 0); SGM_OCV_EVOL
forces one (1 records, 2 planes) or turns the scheme off (0). It applies where the path lanes hold
8 or 16 values (the shapes below are chosen for that: 32-lane lines for 128 < D <= 256, 64-lane
lines for D > 256, SGM_OCV_LPL=16 for D <= 128) and, with the fused vertical WTA, for D > 256.
Every case is compared bit for bit with the oracle (oracle/sgm_oracle.c) in both layouts, with
the scheme off, and at P2 = 255 / 511 (the largest 8- and 9-bit deficits) and 512 (scheme off).
"""
import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu

# (h, w, minD, D, block, lpl16): the path lanes hold 8 or 16 values in each
GEOMS = [
    (40, 330, 3, 144, 5, False),        # 32-lane lines, 8 values per lane
    (36, 420, -5, 96, 7, True),         # 16-lane lines, 8 values
    (30, 520, 0, 256, 9, True),         # 16-lane lines, 16 values
    (28, 700, 20, 320, 11, False),      # 64-lane lines, 8 values (D > 256: the fused vertical WTA reads them too)
    (33, 760, 147, 480, 21, False),     # the shipped D, minD and block
]


@pytest.mark.parametrize("evol", ["0", "1", "2"], ids=["off", "records", "planes"])
@pytest.mark.parametrize("vwta", ["0", "1"], ids=["wta16", "vwta"])
@pytest.mark.parametrize("mode", [0, 1], ids=["SGBM", "HH"])
@pytest.mark.parametrize("geom", GEOMS, ids=[f"{g[0]}x{g[1]}-m{g[2]}-D{g[3]}-b{g[4]}" for g in GEOMS])
def test_evol_match(engine, oracle, synth, pkg, monkeypatch, geom, mode, vwta, evol):
    h, w, minD, D, block, lpl16 = geom
    monkeypatch.setenv("SGM_OCV_EVOL", evol)
    monkeypatch.setenv("SGM_OCV_VWTA", vwta)
    if lpl16:
        monkeypatch.setenv("SGM_OCV_LPL", "16")
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=h * w + D + mode)
    p = pkg.default_params(mode, min_disparity=minD, num_disparities=D, block_size=block, uniqueness_ratio=5,
                           speckle_window_size=0)
    assert p.p2 <= 511
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("compat", [7, 4, 0], ids=["melodic", "lane-tie", "scalar"])
@pytest.mark.parametrize("p1p2", [(10, 255), (200, 511), (200, 512), (0, 400)],
                         ids=["P2-255", "P2-511", "P2-512-off", "P1-0"])
@pytest.mark.parametrize("mode", [0, 1], ids=["SGBM", "HH"])
def test_evol_penalties(engine, oracle, synth, pkg, monkeypatch, mode, p1p2, compat):
    """Deficits at their 9-bit limit (P2 = 511: e reaches 511), the 8-bit boundary, the first P2
    that turns the scheme off, on the shipped D=480 geometry through the fused vertical WTA and
    on D=144 through the row WTA."""
    p1, p2 = p1p2
    for (h, w, minD, D, block), vwta in (((30, 760, 147, 480, 21), "1"), ((40, 330, 3, 144, 5), "0")):
        monkeypatch.setenv("SGM_OCV_VWTA", vwta)
        left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=D + p2 + mode)
        p = pkg.default_params(mode, min_disparity=minD, num_disparities=D, block_size=block, p1=p1, p2=p2,
                               ocv_compat=compat, uniqueness_ratio=3, speckle_window_size=0)
        engine.set_params(p)
        got = engine.match(left, right)
        ref = oracle.match(to_oracle_params(oracle, p), left, right)
        assert np.array_equal(got, ref), f"D {D}: {(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("mode", [0, 1], ids=["SGBM", "HH"])
def test_evol_1080p_both_layouts(engine, synth, pkg, monkeypatch, mode):
    """1920x1080 D=128 (planes by default) and forced records give the int16-volume result."""
    left, right, _ = synth.stereo_pair(1080, 1920, 0, 128, seed=77 + mode)
    p = pkg.default_params(mode, min_disparity=0, num_disparities=128, block_size=5, speckle_window_size=0)
    engine.set_params(p)
    outs = {}
    for evol in ("0", "1", "2"):
        monkeypatch.setenv("SGM_OCV_EVOL", evol)
        outs[evol] = engine.match(left, right)
    assert np.array_equal(outs["1"], outs["0"]), f"records: {(outs['1'] != outs['0']).sum()} pixels differ"
    assert np.array_equal(outs["2"], outs["0"]), f"planes: {(outs['2'] != outs['0']).sum()} pixels differ"


# 64-lane lines of 16 values (512 < D <= 1024) and of 8 (256 < D <= 512, their own kernel instantiation).
# With SGM_OCV_NO_BUF=1 the packed step rebases its
# buffer descriptors on each step's cell — the form every frame whose volumes pass 4 GB takes (the
# processing launch's D = 752 at 2448 x 2048: 5.2 GB) — and, under the fused vertical WTA, stores
# deficit records (vwta 0: the row WTA k_ocv_wta64 reads int16 L, so no deficits there).
REB_GEOMS = [(26, 900, 0, 752, 21), (22, 800, 7, 640, 9), (20, 1150, -3, 1024, 5), (24, 700, 0, 528, 15),
             (28, 700, 20, 320, 11), (26, 760, 0, 512, 21)]     # 8 values per lane: the REBK kernel


@pytest.mark.parametrize("nobuf", ["0", "1"], ids=["offsets", "rebased"])
@pytest.mark.parametrize("evol", ["default", "0"], ids=["evol", "evol-off"])
@pytest.mark.parametrize("vwta", ["0", "1"], ids=["wta64", "vwta"])
@pytest.mark.parametrize("mode", [0, 1], ids=["SGBM", "HH"])
@pytest.mark.parametrize("geom", REB_GEOMS, ids=[f"{g[0]}x{g[1]}-m{g[2]}-D{g[3]}-b{g[4]}" for g in REB_GEOMS])
def test_wide_disparity_rebased_paths(engine, oracle, synth, pkg, monkeypatch, geom, mode, vwta, evol, nobuf):
    h, w, minD, D, block = geom
    if evol != "default":
        monkeypatch.setenv("SGM_OCV_EVOL", evol)
    monkeypatch.setenv("SGM_OCV_VWTA", vwta)
    monkeypatch.setenv("SGM_OCV_NO_BUF", nobuf)
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=h * w + D + mode)
    p = pkg.default_params(mode, min_disparity=minD, num_disparities=D, block_size=block, uniqueness_ratio=2,
                           speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("uniq", [0, 100])
@pytest.mark.parametrize("mode", [0, 1], ids=["SGBM", "HH"])
def test_wide_disparity_rebased_uniqueness_edges(engine, oracle, synth, pkg, monkeypatch, mode, uniq):
    """uniqueness 100 routes the fused vertical WTA to its int form (k_ocv_vwta) over the same
    deficit records; 0 keeps the packed one."""
    monkeypatch.setenv("SGM_OCV_VWTA", "1")
    monkeypatch.setenv("SGM_OCV_NO_BUF", "1")
    left, right, _ = synth.stereo_pair(24, 880, 0, 752, seed=752 + mode + uniq)
    p = pkg.default_params(mode, min_disparity=0, num_disparities=752, block_size=21, uniqueness_ratio=uniq,
                           speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
