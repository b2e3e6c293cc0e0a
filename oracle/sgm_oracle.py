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
        "speckle_range", "subpixel", "lr_check", "median")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


def make_params(mode=MODE_CENSUS8, **kw):
    """Defaults mirror sgm_default_params(): census = north-star config; OCV = node defaults
    (reference src/generate_disparity.cpp:100-112)."""
    if mode == MODE_CENSUS8:
        d = dict(mode=mode, min_disparity=0, num_disparities=128, block_size=0, p1=10, p2=120,
                 uniqueness_ratio=5, disp12_max_diff=1, prefilter_cap=0, speckle_window_size=0,
                 speckle_range=0, subpixel=1, lr_check=1, median=0)
    else:
        d = dict(mode=mode, min_disparity=9, num_disparities=64, block_size=15, p1=200, p2=400,
                 uniqueness_ratio=15, disp12_max_diff=0, prefilter_cap=31, speckle_window_size=100,
                 speckle_range=4, subpixel=1, lr_check=1, median=1)
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
