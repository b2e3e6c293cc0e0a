"""CPU: the rectification restatements in oracle/sgm_oracle.py (initUndistortRectifyMap
CV_32FC1 + remap INTER_CUBIC / BORDER_CONSTANT, generate_disparity.cpp:370-386) against
scalar evaluations written straight from OpenCV's loops, and the library's host-built
INTER_CUBIC table against the oracle's. Parity with OpenCV itself is unpinned: OpenCV is
absent from the image and the reference holds no rectified fixtures."""
import numpy as np
import pytest


def calib(seed=0, w=640, h=480, rot=True):
    """A plausible plumb_bob CameraInfo: K, D(5), R (small rotation), P."""
    rng = np.random.default_rng(seed)
    f = 0.9 * w
    K = np.array([[f, 0, w / 2 + 3.3], [0, f * 1.01, h / 2 - 2.1], [0, 0, 1]], np.float64)
    D = np.array([-0.21, 0.07, 0.0012, -0.0009, -0.011])
    if rot:
        a = rng.normal(0, 0.02, 3)
        th = np.linalg.norm(a)
        k = a / th
        Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        R = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    else:
        R = np.eye(3)
    P = np.array([[f * 0.98, 0, w / 2 - 5.0, -0.12 * f], [0, f * 0.98, h / 2 + 1.5, 0], [0, 0, 1, 0]], np.float64)
    return K, D, R, P


def scalar_map(K, D, R, P, w, h, oracle):
    """initUndistortRectifyMap's scalar loop in Python floats (IEEE double, one rounding per op)."""
    ir = oracle.rectify_inverse(K, P, R)
    k1, k2, p1, p2, k3, k4, k5, k6, s1, s2, s3, s4 = oracle.dist_coeffs(D)
    u0, v0, fx, fy = K[0, 2], K[1, 2], K[0, 0], K[1, 1]
    mx = np.empty((h, w), np.float32)
    my = np.empty((h, w), np.float32)
    for i in range(h):
        _x, _y, _w = i * ir[1] + ir[2], i * ir[4] + ir[5], i * ir[7] + ir[8]
        for j in range(w):
            ww = 1.0 / _w
            x, y = _x * ww, _y * ww
            x2, y2 = x * x, y * y
            r2, _2xy = x2 + y2, 2 * x * y
            kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
            xd = x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2
            yd = y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2
            t0 = 0.0 + 1.0 * xd + 0.0 * yd + 0.0 * 1.0
            t1 = 0.0 + 0.0 * xd + 1.0 * yd + 0.0 * 1.0
            t2 = 0.0 + 0.0 * xd + 0.0 * yd + 1.0 * 1.0
            inv = 1.0 / t2 if t2 else 1.0
            mx[i, j] = np.float32(fx * inv * t0 + u0)
            my[i, j] = np.float32(fy * inv * t1 + v0)
            _x += ir[0]
            _y += ir[3]
            _w += ir[6]
    return mx, my


def scalar_remap(src, mx, my, tab):
    """remapBicubic's branch structure (interior / border / all-outside) for u8, cval = 0."""
    sh, sw = src.shape
    h, w = mx.shape
    out = np.zeros((h, w), np.uint8)
    for y in range(h):
        for x in range(w):
            def rnd(v):
                v = np.float32(v) * np.float32(32)
                if not (-2147483648.0 < v < 2147483648.0):
                    return -2147483648
                return int(np.rint(v))
            X, Y = rnd(mx[y, x]), rnd(my[y, x])
            wt = tab[(Y & 31) * 32 + (X & 31)].astype(np.int64)
            sx = max(-32768, min(32767, X >> 5)) - 1
            sy = max(-32768, min(32767, Y >> 5)) - 1
            if 0 <= sx < max(sw - 3, 0) and 0 <= sy < max(sh - 3, 0):
                s = sum(int(src[sy + a, sx + b]) * int(wt[a * 4 + b]) for a in range(4) for b in range(4))
            elif sx >= sw or sx + 4 <= 0 or sy >= sh or sy + 4 <= 0:
                out[y, x] = 0
                continue
            else:
                s = 0
                for a in range(4):
                    yy = sy + a
                    if not 0 <= yy < sh:
                        continue
                    for b in range(4):
                        xx = sx + b
                        if 0 <= xx < sw:
                            s += int(src[yy, xx]) * int(wt[a * 4 + b])
            out[y, x] = min(max((s + (1 << 14)) >> 15, 0), 255)
    return out


def test_cubic_table_properties(oracle):
    t = oracle.cubic_table()
    assert t.shape == (1024, 16)
    assert (t.astype(np.int64).sum(1) == 32768).all()
    # integer position: the centre weight 1.0 saturates to 32767 and the missing 1 lands on
    # tap (2, 2) — identity remaps still copy exactly (see test_remap_identity)
    assert t[0, 5] == 32767 and t[0, 10] == 1 and np.count_nonzero(t[0]) == 2
    # half-pixel in both axes: symmetric 4x4 kernel of the cubic weights (-0.09375, 0.59375)
    assert t[16 * 32 + 16, 5] == 11552 and t[16 * 32 + 16, 0] == 288


def test_library_cubic_table_matches_oracle(oracle, pkg):
    assert np.array_equal(pkg.cubic_table(), oracle.cubic_table())


def test_remap_identity(oracle):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    mx, my = np.meshgrid(np.arange(53, dtype=np.float32), np.arange(37, dtype=np.float32))
    assert np.array_equal(oracle.remap_cubic(img, mx, my), img)
    # integer shift by (+3, -2): shifted image, zeros where the source is outside
    got = oracle.remap_cubic(img, mx + 3, my - 2)
    ref = np.zeros_like(img)
    ref[2:, :50] = img[:35, 3:]
    assert np.array_equal(got, ref)


def test_remap_matches_scalar_loop(oracle):
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, (23, 31), dtype=np.uint8)
    h, w = 19, 27
    mx = rng.uniform(-6, 37, (h, w)).astype(np.float32)
    my = rng.uniform(-6, 29, (h, w)).astype(np.float32)
    mx[0, :4] = [np.nan, np.inf, -1e12, 3.015625]     # saturating conversions, a 1/64 tie
    my[1, :2] = [1e30, 0.515625]
    tab = oracle.cubic_table()
    assert np.array_equal(oracle.remap_cubic(src, mx, my, tab), scalar_remap(src, mx, my, tab))


@pytest.mark.parametrize("nd", [0, 4, 5, 8, 12])
def test_rectify_map_matches_scalar_loop(oracle, nd):
    K, D, R, P = calib(seed=nd, w=40, h=30)
    Dn = np.concatenate([D, [0.01, -0.002, 0.0005, 0.001, -0.0007, 0.0003, 0.0002]])[:nd]
    mx, my = oracle.rectify_map(K, Dn, R, P, 40, 30)
    sx, sy = scalar_map(K, Dn, R, P, 40, 30, oracle)
    assert np.array_equal(mx.view(np.uint32), sx.view(np.uint32))
    assert np.array_equal(my.view(np.uint32), sy.view(np.uint32))


def test_rectify_map_identity_calibration(oracle):
    K = np.array([[500.0, 0, 320], [0, 500, 240], [0, 0, 1]])
    P = np.hstack([K, np.zeros((3, 1))])
    mx, my = oracle.rectify_map(K, None, None, P, 64, 48)
    gx, gy = np.meshgrid(np.arange(64), np.arange(48))
    assert np.abs(mx - gx).max() < 1e-3 and np.abs(my - gy).max() < 1e-3


def test_rectify_map_rejects_bad_distortion(oracle):
    with pytest.raises(ValueError):
        oracle.dist_coeffs(np.zeros(14))
