"""CPU: the depth / DisparityImage restatements in oracle/sgm_oracle.py against scalar
float32 evaluations written straight from the reference's loops, and calc_q through the
C-ABI (host-only function) against the oracle."""
import numpy as np
import pytest

f32 = np.float32


def _scalar_depth(d, Q, zmin, zmax):
    """disparity_to_depth.cpp:148-205, one float32 operation at a time."""
    wz, q03, q13, q32, q33 = f32(Q[2, 3]), f32(Q[0, 3]), f32(Q[1, 3]), f32(Q[3, 2]), f32(Q[3, 3])
    h, w = d.shape
    depth = np.zeros((h, w), np.float32)
    pts = []
    with np.errstate(all="ignore"):
        for i in range(h):
            for j in range(w):
                v = f32(d[i, j])
                if v != 0 and v != f32(10000):
                    ww = f32(f32(v * q32) + q33)
                    x = f32(f32(f32(j) + q03) / ww)
                    y = f32(f32(f32(i) + q13) / ww)
                    z = f32(wz / ww)
                    if ww > 0 and z > 0 and float(z) <= zmax and float(z) >= zmin:
                        depth[i, j] = z
                        pts.append((x, y, z))
    return depth, np.array(pts, np.float32).reshape(-1, 3)


def _sample_disp(rng, h, w):
    d = (rng.integers(-40, 2000, (h, w)) / 16.0).astype(np.float32)
    d[rng.random((h, w)) < 0.1] = 0
    d[rng.random((h, w)) < 0.1] = 10000
    return d


def _q():
    K = np.array([[712.5, 0, 331.2], [0, 712.5, 247.9], [0, 0, 1]])
    Pl = np.array([[712.5, 0, 331.2, 0], [0, 712.5, 247.9, 0], [0, 0, 1, 0]])
    Pr = Pl.copy()
    Pr[0, 3] = -712.5 * 0.119
    Pr[0, 2] = 329.8
    return K, Pr, Pl


def test_depth_oracle_matches_scalar_loop(oracle):
    rng = np.random.default_rng(5)
    d = _sample_disp(rng, 23, 37)
    K, Pr, Pl = _q()
    Q = oracle.calc_q(K, Pr, Pl)
    for zmin, zmax in [(0.0, 100.0), (0.5, 3.0)]:
        depth, pts, rgba = oracle.depth_points(d, Q, zmin, zmax)
        sd, sp = _scalar_depth(d, Q, zmin, zmax)
        assert np.array_equal(depth.view(np.uint32), sd.view(np.uint32))
        assert np.array_equal(pts.view(np.uint32), sp.view(np.uint32))
        assert (rgba == 0xFF000000).all()


def test_depth_oracle_colors(oracle):
    rng = np.random.default_rng(6)
    d = _sample_disp(rng, 9, 11)
    Q = oracle.calc_q(*_q())
    mono = rng.integers(0, 256, (9, 11), dtype=np.uint8)
    bgr = rng.integers(0, 256, (9, 11, 3), dtype=np.uint8)
    _, _, r1 = oracle.depth_points(d, Q, 0, 100, mono)
    depth, _, r3 = oracle.depth_points(d, Q, 0, 100, bgr)
    ok = depth.ravel() > 0
    m = mono.ravel()[ok].astype(np.uint32)
    assert np.array_equal(r1, 0xFF000000 | (m << 16) | (m << 8) | m)
    c = bgr.reshape(-1, 3)[ok].astype(np.uint32)
    assert np.array_equal(r3, 0xFF000000 | (c[:, 2] << 16) | (c[:, 1] << 8) | c[:, 0])


def test_disparity_to_msg_oracle(oracle):
    rng = np.random.default_rng(7)
    d16 = rng.integers(-200, 4000, (13, 17)).astype(np.int16)
    out = oracle.disparity_to_msg(d16, 1.5, 200.25)
    for i in range(13):
        for j in range(17):
            v = f32(d16[i, j]) * f32(0.0625)
            if v < f32(1.5) or v > f32(200.25):
                v = f32(10000)
            assert out[i, j] == v


def test_calc_q_cabi_matches_oracle(pkg, oracle):
    K, Pr, Pl = _q()
    assert np.array_equal(pkg.calc_q(K, Pr, Pl), oracle.calc_q(K, Pr, Pl))
    Q = oracle.calc_q(K, Pr, Pl)
    assert Q[2, 3] == 712.5 and Q[0, 3] == -331.2 and Q[3, 2] == pytest.approx(1 / 0.119)
