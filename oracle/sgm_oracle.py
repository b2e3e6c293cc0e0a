"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/sgm_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
It is the checker, never the thing measured or shipped: the product path is
libsgm_hip.so (i3dr_stereo_camera-ros_amd/csrc) and never loads this library.

Parity status: **parity unpinned** against real OpenCV (absent from the image; the
reference holds no tests or fixtures — SURVEY.md §8c). See sgm_oracle.c's header.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libsgm_oracle.so")

MODE_OCV_SGBM5 = 0
MODE_OCV_HH8 = 1
MODE_CENSUS8 = 2

DIRS = [(0, 1), (0, -1), (1, 1), (-1, 1), (1, -1), (-1, -1), (1, 0), (-1, 0)]


class SgmParams(ctypes.Structure):
    """Mirror of `sgm_params` (include/sgm_hip.h)."""
    _fields_ = [(n, ctypes.c_int) for n in (
        "mode", "min_disparity", "num_disparities", "block_size", "p1", "p2",
        "uniqueness_ratio", "disp12_max_diff", "prefilter_cap", "speckle_window_size",
        "speckle_range", "subpixel", "lr_check", "median", "ocv_compat")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


def make_params(mode=MODE_CENSUS8, **kw):
    """Defaults mirror sgm_default_params(): census = north-star config; OCV = node defaults
    (reference src/generate_disparity.cpp:100-112) with ocv_compat = COMPAT_MELODIC (the
    OpenCV 3.2 SSE2 build of the reference's Dockerfile:1)."""
    if mode == MODE_CENSUS8:
        d = dict(mode=mode, min_disparity=0, num_disparities=128, block_size=0, p1=10, p2=120,
                 uniqueness_ratio=5, disp12_max_diff=1, prefilter_cap=0, speckle_window_size=0,
                 speckle_range=0, subpixel=1, lr_check=1, median=0, ocv_compat=0)
    else:
        d = dict(mode=mode, min_disparity=9, num_disparities=64, block_size=15, p1=200, p2=400,
                 uniqueness_ratio=15, disp12_max_diff=0, prefilter_cap=31, speckle_window_size=100,
                 speckle_range=4, subpixel=1, lr_check=1, median=1, ocv_compat=COMPAT_MELODIC)
    d.update(kw)
    p = SgmParams()
    for k, v in d.items():
        setattr(p, k, int(v))
    return p


def build(force=False):
    """Compile the oracle with gcc (test infrastructure build, also run by build())."""
    src = os.path.join(HERE, "sgm_oracle.c")
    if not force and os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= max(
            os.path.getmtime(src), os.path.getmtime(os.path.join(ROOT, "include", "sgm_hip.h"))):
        return LIB_PATH
    cmd = ["gcc", "-O3", "-march=x86-64-v2", "-fopenmp", "-fPIC", "-shared", "-Wall",
           "-I" + os.path.join(ROOT, "include"), src, "-o", LIB_PATH]
    subprocess.check_call(cmd)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        u8p, i16p, u16p, u64p = (ctypes.c_void_p,) * 4
        L.sgmref_match.argtypes = [P(SgmParams), u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                   i16p, ctypes.c_size_t]
        L.sgmref_census9x7.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, u64p]
        L.sgmref_census_path.argtypes = [P(SgmParams), u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                         ctypes.c_int, u8p]
        L.sgmref_census_sum.argtypes = [P(SgmParams), u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, u16p]
        L.sgmref_ocv_cost.argtypes = [P(SgmParams), u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, i16p]
        L.sgmref_wta.argtypes = [P(SgmParams), ctypes.c_int, ctypes.c_int, u16p, i16p, ctypes.c_size_t]
        L.sgmref_median3.argtypes = [i16p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t]
        L.sgmref_filter_speckles.argtypes = [i16p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.sgmref_effective.argtypes = [P(SgmParams), ctypes.c_int, ctypes.c_int, P(ctypes.c_int)]
        L.sgmref_set_ocv_compat.argtypes = [ctypes.c_int]
        L.sgmref_get_ocv_compat.restype = ctypes.c_int
        L.sgmref_num_threads.restype = ctypes.c_int
        L.sgmref_set_num_threads.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"oracle {what} failed with status {rc}")


def effective(p, w, h):
    out = (ctypes.c_int * 16)()
    _check(lib().sgmref_effective(ctypes.byref(p), w, h, out), "effective")
    keys = ["minD", "D", "SW2", "SH2", "ftzero", "uniq", "disp12", "P1", "P2", "minX1", "maxX1",
            "width1", "invalid", "subpix", "lr", "median"]
    return dict(zip(keys, list(out)))


def match(p, left, right):
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    h, w = left.shape
    disp = np.empty((h, w), np.int16)
    _check(lib().sgmref_match(ctypes.byref(p), _ptr(left), _ptr(right), w, h, w, _ptr(disp), w), "match")
    return disp


def census(img):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.empty((h, w), np.uint64)
    _check(lib().sgmref_census9x7(_ptr(img), w, h, w, _ptr(out)), "census")
    return out


def census_path(p, left, right, direction):
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    h, w = left.shape
    e = effective(p, w, h)
    vol = np.zeros((h, max(e["width1"], 0), e["D"]), np.uint8)
    _check(lib().sgmref_census_path(ctypes.byref(p), _ptr(left), _ptr(right), w, h, w, direction, _ptr(vol)),
           "census_path")
    return vol


def census_sum(p, left, right):
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    h, w = left.shape
    e = effective(p, w, h)
    S = np.zeros((h, max(e["width1"], 0), e["D"]), np.uint16)
    _check(lib().sgmref_census_sum(ctypes.byref(p), _ptr(left), _ptr(right), w, h, w, _ptr(S)), "census_sum")
    return S


def ocv_cost(p, left, right):
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    h, w = left.shape
    e = effective(p, w, h)
    C = np.zeros((h, max(e["width1"], 0), e["D"]), np.int16)
    _check(lib().sgmref_ocv_cost(ctypes.byref(p), _ptr(left), _ptr(right), w, h, w, _ptr(C)), "ocv_cost")
    return C


def wta(p, S, w):
    S = np.ascontiguousarray(S, np.uint16)
    h = S.shape[0]
    disp = np.empty((h, w), np.int16)
    _check(lib().sgmref_wta(ctypes.byref(p), w, h, _ptr(S), _ptr(disp), w), "wta")
    return disp


def median3(disp):
    d = np.ascontiguousarray(disp, np.int16).copy()
    h, w = d.shape
    _check(lib().sgmref_median3(_ptr(d), w, h, w), "median3")
    return d


def filter_speckles(disp, new_val, max_size, max_diff):
    d = np.ascontiguousarray(disp, np.int16).copy()
    h, w = d.shape
    _check(lib().sgmref_filter_speckles(_ptr(d), w, h, w, new_val, max_size, max_diff), "speckles")
    return d


# OpenCV build variants of the OCV modes (sgm_oracle.c); 0 = the default
# restatement the GPU engine reproduces.
OCV_COL0_LEGACY = 1    # 3.x: the vertical running sum skips C' column 0 for y > 0
OCV_SIMD_SAT = 2       # CV_SIMD branches: int16 saturating sums / recurrence / S
OCV_LANE_TIE = 4       # MODE_SGBM SSE2 WTA: lowest lane (d mod 8) wins among equal minima
COMPAT_SCALAR = 0                                          # the scalar 4.x restatement
COMPAT_NOETIC = OCV_SIMD_SAT                               # noetic x86-64: OpenCV 4.2 SIMD
COMPAT_MELODIC = OCV_COL0_LEGACY | OCV_SIMD_SAT | OCV_LANE_TIE  # melodic x86-64: OpenCV 3.2 SSE2


class ocv_compat:
    """Context manager: run the oracle's OCV modes with the given SGMREF_OCV_* bits."""

    def __init__(self, flags):
        self.flags = int(flags)

    def __enter__(self):
        self.prev = int(lib().sgmref_get_ocv_compat())
        lib().sgmref_set_ocv_compat(self.flags)
        return self

    def __exit__(self, *a):
        lib().sgmref_set_ocv_compat(self.prev)


def set_threads(n):
    lib().sgmref_set_num_threads(int(n))


def num_threads():
    return int(lib().sgmref_num_threads())


# ---------------------------------------------------------------------------------------
# After the matcher: numpy float32 restatements. numpy applies
# one IEEE rounding per float32 operation (no fused multiply-add), the same as the
# reference's scalar C++ expressions; parity with the GPU is bit-exact.
# ---------------------------------------------------------------------------------------
MISSING_Z = np.float32(10000.0)      # image_geometry::StereoCameraModel::MISSING_Z


def disparity_to_msg(disp16, min_disparity, max_disparity):
    """generate_disparity.cpp:426-452: convertTo(dmat, CV_32F, 1/16), then
    setTo(MISSING_Z, dmat < min_disparity) and setTo(MISSING_Z, dmat > max_disparity)."""
    d = np.asarray(disp16, np.int16).astype(np.float32) * np.float32(0.0625)
    d[d < np.float32(min_disparity)] = MISSING_Z
    d[d > np.float32(max_disparity)] = MISSING_Z
    return d


def calc_q(K, P_right, P_left):
    """disparity_to_depth.cpp:62-84 (doubles)."""
    K = np.asarray(K, np.float64).reshape(3, 3)
    Pr = np.asarray(P_right, np.float64).reshape(3, 4)
    Pl = np.asarray(P_left, np.float64).reshape(3, 4)
    cx, cxr, cy, fx = Pl[0, 2], Pr[0, 2], Pl[1, 2], K[0, 0]
    T = -Pr[0, 3] / fx
    q = np.zeros((4, 4), np.float64)
    q[0, 0] = 1.0
    q[0, 3] = -cx
    q[1, 1] = 1.0
    q[1, 3] = -cy
    q[2, 3] = fx
    q[3, 2] = 1.0 / T
    q[3, 3] = -(cx - cxr) / T
    return q


def depth_points(disp, Q, depth_min, depth_max, color=None):
    """disparity_to_depth.cpp:127-205: depth image and the XYZRGB points in push_back
    (raster) order. Q(2,3), Q(0,3), Q(1,3), Q(3,2), Q(3,3) are cast to float (:134-138); the
    depth window is compared in double (z promoted). color: None, HxW (MONO8) or HxWx3 (BGR8).
    Returns (depth float32 HxW, points float32 Nx3, rgba uint32 N)."""
    d = np.asarray(disp, np.float32)
    h, w = d.shape
    Q = np.asarray(Q, np.float64)
    wz, q03, q13, q32, q33 = (np.float32(Q[2, 3]), np.float32(Q[0, 3]), np.float32(Q[1, 3]),
                              np.float32(Q[3, 2]), np.float32(Q[3, 3]))
    jj = np.broadcast_to(np.arange(w, dtype=np.float32)[None, :], (h, w))
    ii = np.broadcast_to(np.arange(h, dtype=np.float32)[:, None], (h, w))
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        ww = d * q32 + q33                      # two float32 roundings, like the C++ expression
        x = (jj + q03) / ww
        y = (ii + q13) / ww
        z = wz / ww
        ok = (d != 0) & (d != MISSING_Z) & (ww > 0) & (z > 0)
        z64 = z.astype(np.float64)
        ok &= (z64 <= float(depth_max)) & (z64 >= float(depth_min))
    depth = np.where(ok, z, np.float32(0)).astype(np.float32)
    sel = np.nonzero(ok.ravel())[0]
    pts = np.stack([x.ravel()[sel], y.ravel()[sel], z.ravel()[sel]], axis=1).astype(np.float32)
    if color is None:
        b = g = r = np.zeros(len(sel), np.uint32)
    else:
        c = np.asarray(color, np.uint8)
        if c.ndim == 2:
            b = g = r = c.ravel()[sel].astype(np.uint32)
        else:
            cc = c.reshape(-1, 3)[sel].astype(np.uint32)
            b, g, r = cc[:, 0], cc[:, 1], cc[:, 2]
    rgba = (np.uint32(0xFF000000) | (r << 16) | (g << 8) | b).astype(np.uint32)
    return depth, pts, rgba


# ---------------------------------------------------------------------------------------
# Rectification: the node's rectify() — cv::initUndistortRectifyMap
# (CV_32FC1 maps) + cv::remap(INTER_CUBIC, BORDER_CONSTANT 0) — generate_disparity.cpp:370-386,
# rectify.cpp:111-127. OpenCV is absent from the image: this restates its published scalar
# algorithm (imgproc undistort.cpp / imgwarp.cpp), **parity unpinned** (no fixture holds a
# rectified image). float32 / float64 numpy arithmetic, one IEEE rounding per operation.
# ---------------------------------------------------------------------------------------
INTER_BITS = 5
INTER_TAB_SIZE = 1 << INTER_BITS          # 32 sub-pixel positions per axis
INTER_REMAP_COEF_BITS = 15
INTER_REMAP_COEF_SCALE = 1 << INTER_REMAP_COEF_BITS


def _cubic_coeffs(x):
    """imgwarp.cpp interpolateCubic (float, A = -0.75)."""
    f = np.float32
    A, x = f(-0.75), f(x)
    one = f(1)
    c0 = ((A * (x + one) - f(5) * A) * (x + one) + f(8) * A) * (x + one) - f(4) * A
    c1 = ((A + f(2)) * x - (A + f(3))) * x * x + one
    c2 = ((A + f(2)) * (one - x) - (A + f(3))) * (one - x) * (one - x) + one
    c3 = one - c0 - c1 - c2
    return [c0, c1, c2, c3]


def cubic_table():
    """initInterTab2D(INTER_CUBIC, fixpt=true): int16 [32*32][16] weights, entry (fy*32 + fx),
    tap k1*4 + k2 = row sy-1+k1, column sx-1+k2. The float products are rounded to 1/32768
    (cvRound: half to even); an entry whose sum misses 32768 gets the difference on the
    largest (sum < 32768) / smallest (sum > 32768) tap of rows/columns 2..3."""
    scale = np.float32(1.0) / np.float32(INTER_TAB_SIZE)
    t1 = [_cubic_coeffs(np.float32(i) * scale) for i in range(INTER_TAB_SIZE)]
    tab = np.zeros((INTER_TAB_SIZE * INTER_TAB_SIZE, 16), np.int16)
    for i in range(INTER_TAB_SIZE):
        for j in range(INTER_TAB_SIZE):
            it = [0] * 16
            for k1 in range(4):
                vy = t1[i][k1]
                for k2 in range(4):
                    v = np.float32(vy * t1[j][k2])
                    r = int(np.rint(np.float32(v * np.float32(INTER_REMAP_COEF_SCALE))))
                    it[k1 * 4 + k2] = max(-32768, min(32767, r))
            isum = sum(it)
            if isum != INTER_REMAP_COEF_SCALE:
                diff = isum - INTER_REMAP_COEF_SCALE
                k0 = 2
                Mk1 = Mk2 = mk1 = mk2 = k0
                for k1 in range(k0, k0 + 2):
                    for k2 in range(k0, k0 + 2):
                        if it[k1 * 4 + k2] < it[mk1 * 4 + mk2]:
                            mk1, mk2 = k1, k2
                        elif it[k1 * 4 + k2] > it[Mk1 * 4 + Mk2]:
                            Mk1, Mk2 = k1, k2
                if diff < 0:
                    it[Mk1 * 4 + Mk2] -= diff
                else:
                    it[mk1 * 4 + mk2] -= diff
            tab[i * INTER_TAB_SIZE + j] = it
    return tab


def rectify_inverse(K, P, R=None):
    """iR = (P[:, :3] * R)^-1 of initUndistortRectifyMap: the 3x3 product summed k = 0..2 in
    order, the inverse by cv::invert's 3x3 closed form (DECOMP_LU: adjugate * (1 / det3))."""
    Ar = np.asarray(P, np.float64).reshape(3, -1)[:, :3]
    R = np.eye(3) if R is None else np.asarray(R, np.float64).reshape(3, 3)
    M = np.zeros((3, 3))
    for i in range(3):
        for j in range(3):
            s = 0.0
            for k in range(3):
                s += Ar[i, k] * R[k, j]
            M[i, j] = s
    m = M
    det = (m[0, 0] * (m[1, 1] * m[2, 2] - m[1, 2] * m[2, 1]) -
           m[0, 1] * (m[1, 0] * m[2, 2] - m[1, 2] * m[2, 0]) +
           m[0, 2] * (m[1, 0] * m[2, 1] - m[1, 1] * m[2, 0]))
    if det == 0.0:
        raise ValueError("singular P[:, :3] * R")
    d = 1.0 / det
    t = [(m[1, 1] * m[2, 2] - m[1, 2] * m[2, 1]) * d,
         (m[0, 2] * m[2, 1] - m[0, 1] * m[2, 2]) * d,
         (m[0, 1] * m[1, 2] - m[0, 2] * m[1, 1]) * d,
         (m[1, 2] * m[2, 0] - m[1, 0] * m[2, 2]) * d,
         (m[0, 0] * m[2, 2] - m[0, 2] * m[2, 0]) * d,
         (m[0, 2] * m[1, 0] - m[0, 0] * m[1, 2]) * d,
         (m[1, 0] * m[2, 1] - m[1, 1] * m[2, 0]) * d,
         (m[0, 1] * m[2, 0] - m[0, 0] * m[2, 1]) * d,
         (m[0, 0] * m[1, 1] - m[0, 1] * m[1, 0]) * d]
    return np.array(t, np.float64)


def dist_coeffs(D):
    """OpenCV's 4/5/8/12-element distortion vector -> k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4."""
    D = [] if D is None else [float(v) for v in np.asarray(D, np.float64).ravel()]
    if len(D) not in (0, 4, 5, 8, 12):
        raise ValueError("distortion vector must have 0, 4, 5, 8 or 12 elements")
    return np.array(D + [0.0] * (12 - len(D)), np.float64)


def rectify_map(K, D, R, P, width, height):
    """initUndistortRectifyMap(K, D, R, P, (W, H), CV_32FC1) — the scalar loop: per row i,
    _x = i*ir1 + ir2 (etc.), advanced by += ir0 per column; per pixel the rational + tangential
    + thin-prism model, identity tilt, u = fx*invProj*xt + u0, stored as float.
    Returns (map_x, map_y) float32 HxW."""
    K = np.asarray(K, np.float64).reshape(3, 3)
    ir = rectify_inverse(K, P, R)
    k1, k2, p1, p2, k3, k4, k5, k6, s1, s2, s3, s4 = dist_coeffs(D)
    u0, v0, fx, fy = K[0, 2], K[1, 2], K[0, 0], K[1, 1]
    i = np.arange(height, dtype=np.float64)[:, None]

    def run(c_i, c_0, c_j):      # row start i*c_i + c_0, then sequential += c_j
        a = np.empty((height, width), np.float64)
        a[:, :1] = i * c_i + c_0
        a[:, 1:] = c_j
        return np.cumsum(a, axis=1)    # np.add.accumulate: strictly left-to-right
    _x, _y, _w = run(ir[1], ir[2], ir[0]), run(ir[4], ir[5], ir[3]), run(ir[7], ir[8], ir[6])
    with np.errstate(all="ignore"):
        w = 1.0 / _w
        x = _x * w
        y = _y * w
        x2 = x * x
        y2 = y * y
        r2 = x2 + y2
        _2xy = 2 * x * y
        kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
        xd = x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2
        yd = y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2
        # matTilt (identity) * (xd, yd, 1): Matx product, s = 0; s += a(i,k) * b(k)
        t0 = ((0.0 + 1.0 * xd) + 0.0 * yd) + 0.0 * 1.0
        t1 = ((0.0 + 0.0 * xd) + 1.0 * yd) + 0.0 * 1.0
        t2 = ((0.0 + 0.0 * xd) + 0.0 * yd) + 1.0 * 1.0
        inv = np.where(t2 != 0, 1.0 / np.where(t2 != 0, t2, 1.0), 1.0)
        u = fx * inv * t0 + u0
        v = fy * inv * t1 + v0
    return u.astype(np.float32), v.astype(np.float32)


def _round_sat_int(v):
    """saturate_cast<int>(float) = cvRound: half to even; out of range / NaN -> INT_MIN
    (cvtss2si's integer indefinite)."""
    v = np.asarray(v, np.float32)
    ok = (v > np.float32(-2147483648.0)) & (v < np.float32(2147483648.0))
    r = np.rint(np.where(ok, v, 0)).astype(np.int64)
    return np.where(ok, r, -2147483648).astype(np.int64)


def remap_cubic(src, map_x, map_y, tab=None):
    """cv::remap(src, dst, map_x, map_y, INTER_CUBIC, BORDER_CONSTANT, 0) for u8 mono:
    X = cvRound(map_x * 32) -> integer part saturate_cast<short>(X >> 5), fraction X & 31 (same
    for Y); dst = saturate_u8((sum over in-image taps of src * w + 2^14) >> 15), taps outside
    the image read the border value 0."""
    src = np.asarray(src, np.uint8)
    sh, sw = src.shape
    tab = cubic_table() if tab is None else tab
    X = _round_sat_int(np.asarray(map_x, np.float32) * np.float32(INTER_TAB_SIZE))
    Y = _round_sat_int(np.asarray(map_y, np.float32) * np.float32(INTER_TAB_SIZE))
    fxy = (Y & (INTER_TAB_SIZE - 1)) * INTER_TAB_SIZE + (X & (INTER_TAB_SIZE - 1))
    sx = np.clip(X >> INTER_BITS, -32768, 32767) - 1
    sy = np.clip(Y >> INTER_BITS, -32768, 32767) - 1
    w = tab[fxy].astype(np.int64)                   # H x W x 16
    acc = np.zeros(X.shape, np.int64)
    s64 = src.astype(np.int64)
    for k1 in range(4):
        yy = sy + k1
        oky = (yy >= 0) & (yy < sh)
        for k2 in range(4):
            xx = sx + k2
            ok = oky & (xx >= 0) & (xx < sw)
            px = np.where(ok, s64[np.clip(yy, 0, sh - 1), np.clip(xx, 0, sw - 1)], 0)
            acc += px * w[..., k1 * 4 + k2]
    return np.clip((acc + (1 << (INTER_REMAP_COEF_BITS - 1))) >> INTER_REMAP_COEF_BITS, 0, 255).astype(np.uint8)
