"""GPU parity of the packed OpenCV-mode row WTA (csrc/ocv_sgm.hip `k_ocv_wta16_pk`).

In the plain int16 regime (no flagged frame) every path cost lies in [0, 32767], so OpenCV's
saturating sum order (pass 1 saturated, then the fifth path or pass 2) is
min(sum, 32767) in any order. The kernel sums in packed u16 pairs: saturating i16 adds of the
int16 volumes, or, with deficit volumes (Geom::evol, L = C' - e), S = min(NDIR * min(C', Cc) - E,
32767) from the summed deficits E. Uniqueness is the census WTA's sum test (the sum of
max(T - S, 0) against the window's share), the subpixel step branch-free. Every case here is
compared bit for bit with the oracle (oracle/sgm_oracle.c); uniqueness >= 100 keeps k_ocv_wta16.
"""
import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("evol", ["0", "1", "2"], ids=["int16", "records", "planes"])
@pytest.mark.parametrize("mode", [0, 1], ids=["SGBM", "HH"])
@pytest.mark.parametrize("D", [128, 112, 256, 208])
def test_wta_pk_saturated_sums(engine, oracle, pkg, monkeypatch, D, mode, evol):
    """Noise under a 13x13 box: C' up to 169 * 125 + P2 stays in int16 (plain regime, no gate),
    while the sums of five or eight path costs pass 32767 — S saturates for many d, and for the
    deficit volumes C' passes the clamp Cc = ceil((32767 + NDIR * P2) / NDIR)."""
    if evol == "2" and D % 128:
        pytest.skip("planes need D % 128 == 0")
    monkeypatch.setenv("SGM_OCV_EVOL", evol)
    monkeypatch.setenv("SGM_OCV_VWTA", "0")
    monkeypatch.setenv("SGM_OCV_LPL", "16")          # 8 or 16 values per path lane: deficits allowed
    rng = np.random.default_rng(D * 7 + mode)
    h, w = 30, D + 150
    left = rng.integers(0, 256, (h, w), dtype=np.uint8)
    right = rng.integers(0, 256, (h, w), dtype=np.uint8)
    p = pkg.default_params(mode, min_disparity=-2, num_disparities=D, block_size=13, p1=60, p2=480,
                           uniqueness_ratio=4, speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("compat", [7, 0], ids=["melodic", "scalar"])
@pytest.mark.parametrize("uniq", [0, 1, 10, 50, 99, 100, 150])
@pytest.mark.parametrize("D", [32, 64, 128, 160])
def test_wta_pk_uniqueness(engine, oracle, synth, pkg, D, uniq, compat):
    """Every uniqueness ratio class: 0 (no test), small, large, 99 (kq = 1: T = 100 * minS, clamped
    at 32768), and >= 100 (the int kernel); the 3.x lane-tie rule under melodic."""
    left, right, _ = synth.stereo_pair(36, D + 140, 0, D, seed=D + uniq + compat)
    p = pkg.default_params(0, min_disparity=0, num_disparities=D, block_size=5, uniqueness_ratio=uniq,
                           ocv_compat=compat, speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("mode", [0, 1], ids=["SGBM", "HH"])
def test_wta_pk_flat_ties(engine, oracle, pkg, mode):
    """Flat and periodic images: many exact ties of the minimal S across d and lanes (the first-d
    and lane-tie key orders), zero sums (minS = 0, T = 0)."""
    h, w, D = 24, 300, 64
    x = np.arange(w)
    left = np.tile(((x // 3) % 2 * 120 + 60).astype(np.uint8), (h, 1))
    right = np.roll(left, -8, axis=1)
    left[:, :40] = 128
    right[:, :40] = 128
    for compat in (7, 0):
        p = pkg.default_params(mode, min_disparity=0, num_disparities=D, block_size=3, uniqueness_ratio=10,
                               ocv_compat=compat, speckle_window_size=0)
        engine.set_params(p)
        got = engine.match(left, right)
        ref = oracle.match(to_oracle_params(oracle, p), left, right)
        assert np.array_equal(got, ref), f"compat {compat}: {(got != ref).sum()} pixels differ"
