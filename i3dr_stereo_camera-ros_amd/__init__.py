"""MI355X-native SGM disparity engine — Python host mirror of the reference's plugin surface.

The compute path is libsgm_hip.so (hand-written HIP for gfx950, csrc/) behind the C-ABI in
include/sgm_hip.h. This module binds it with ctypes and mirrors, name for name, the
reference's host-side interface for the hot path so tests read like the reference's code:

  * `MatcherHIPSGM`      — AbstractStereoMatcher subclass semantics
                           (reference include/stereoMatcher/abstractStereoMatcher.h:12-92,
                            setters as src/stereoMatcher/matcherOpenCVSGBM.cpp:53-110)
  * `stereo_match`       — generate_disparity.cpp:334-368
  * `process_disparity`  — generate_disparity.cpp:398-456 (x1/16, depth window, MISSING_Z)
  * `parameter_callback` — generate_disparity.cpp:735-845 (cfg sanitising, matcher swap)

There is no CPU fallback: if the HIP library is missing or no device is visible, matching
fails loudly (MatcherHIPSGM.forwardMatch returns -1 exactly like the OpenCV wrapper on an
exception, and `Engine` raises).
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libsgm_hip.so")

ABI_VERSION = 4     # include/sgm_hip.h SGM_ABI_VERSION
MODE_OCV_SGBM5 = 0
MODE_OCV_HH8 = 1
MODE_CENSUS8 = 2

SGM_OK, SGM_ERR_ARG, SGM_ERR_PARAM, SGM_ERR_DEVICE, SGM_ERR_ALLOC, SGM_ERR_UNSUPPORTED = 0, -1, -2, -3, -4, -5

# reference enum (cfg/i3DR_Disparity.cfg:11-17) + the new entry this engine adds
CV_StereoBM, CV_StereoSGBM, I3DR_StereoSGM, CV_StereoBMCuda, CV_StereoBPCuda, CV_StereoCSBPCuda = range(6)
HIP_StereoSGM = 6

MISSING_Z = 10000.0  # image_geometry::StereoCameraModel::MISSING_Z

# sgm_params.ocv_compat: the OpenCV build the OCV modes reproduce (include/sgm_hip.h SGM_OCV_*)
OCV_COL0_LEGACY, OCV_SIMD_SAT, OCV_LANE_TIE = 1, 2, 4
COMPAT_SCALAR = 0                                               # scalar 4.x restatement
COMPAT_NOETIC = OCV_SIMD_SAT                                    # noetic x86-64 (OpenCV 4.2)
COMPAT_MELODIC = OCV_COL0_LEGACY | OCV_SIMD_SAT | OCV_LANE_TIE  # melodic x86-64 (OpenCV 3.2), default
COMPAT_NAMES = {"scalar": COMPAT_SCALAR, "noetic": COMPAT_NOETIC, "melodic": COMPAT_MELODIC}


def ocv_compat_from_env(default=COMPAT_MELODIC):
    """SGM_HIP_OCV_COMPAT = melodic | noetic | scalar | <bits> (the adapters read the same
    variable)."""
    raw = os.environ.get("SGM_HIP_OCV_COMPAT")
    v = (raw or "").strip().lower()
    if not v:
        return default
    if v in COMPAT_NAMES:
        return COMPAT_NAMES[v]
    try:
        return int(v, 0) & 7
    except ValueError:      # the C++ adapter core (hip_sgm_core.cpp) warns and keeps the default too
        sys.stderr.write(f'SGM_HIP_OCV_COMPAT="{raw}" is not melodic | noetic | scalar | <bits>: using {default}\n')
        return default

EXPORTS = [
    "sgm_device_count", "sgm_create", "sgm_destroy", "sgm_default_params", "sgm_set_params", "sgm_get_params",
    "sgm_check_params", "sgm_match", "sgm_match_f32", "sgm_match_device", "sgm_match_device_batch", "sgm_match_batch", "sgm_match_tiled",
    "sgm_match_tiled_device", "sgm_match_tiled_exact", "sgm_abi_version", "sgm_host_register", "sgm_host_unregister", "sgm_synchronize", "sgm_last_error",
    "sgm_set_profiling", "sgm_get_stage_times", "sgm_profiled_matches", "sgm_stage_name", "sgm_stage_bytes",
    "sgm_stage_launches", "sgm_disparity_to_msg", "sgm_calc_q", "sgm_depth_points", "sgm_rectify_map",
    "sgm_remap_cubic", "sgm_cubic_table", "sgm_set_rectification", "sgm_match_device_batch_rect", "sgm_debug_census",
    "sgm_debug_census_path", "sgm_debug_ocv_cost", "sgm_debug_median3", "sgm_debug_speckle", "sgm_debug_path_items",
]


class SgmParams(ctypes.Structure):
    """`sgm_params` of include/sgm_hip.h."""
    _fields_ = [(n, ctypes.c_int) for n in (
        "mode", "min_disparity", "num_disparities", "block_size", "p1", "p2",
        "uniqueness_ratio", "disp12_max_diff", "prefilter_cap", "speckle_window_size",
        "speckle_range", "subpixel", "lr_check", "median", "ocv_compat")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}

    def copy(self, **kw):
        p = SgmParams()
        for n, _ in self._fields_:
            setattr(p, n, getattr(self, n))
        for k, v in kw.items():
            setattr(p, k, int(v))
        return p


_lib = None


def load_library(path=None):
    """Load libsgm_hip.so (SGM_HIP_LIB overrides the in-tree path, e.g. for an experimental
    build); raises if it is missing (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("SGM_HIP_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(f"libsgm_hip.so not found at {path}: run build() / build_ext.py first")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7).
    # Loading torch first makes the dynamic loader bind this library to that same copy, so
    # device pointers and streams from torch are valid here (and torch still finds the GPU).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    P = ctypes.POINTER
    vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.sgm_device_count.restype = ci
    L.sgm_create.argtypes = [P(ctypes.c_void_p), ci]
    L.sgm_destroy.argtypes = [vp]
    L.sgm_destroy.restype = None
    L.sgm_default_params.argtypes = [P(SgmParams), ci]
    L.sgm_default_params.restype = None
    L.sgm_set_params.argtypes = [vp, P(SgmParams)]
    L.sgm_get_params.argtypes = [vp, P(SgmParams)]
    L.sgm_check_params.argtypes = [P(SgmParams), ci, ci]
    L.sgm_match.argtypes = [vp, vp, vp, ci, ci, sz, vp, sz]
    L.sgm_match_f32.argtypes = [vp, vp, vp, ci, ci, sz, vp, sz]
    L.sgm_match_device.argtypes = [vp, vp, vp, ci, ci, sz, vp, sz, vp]
    L.sgm_match_device_batch.argtypes = [vp, P(vp), P(vp), ci, ci, ci, sz, P(vp), sz, vp]
    L.sgm_match_batch.argtypes = [vp, P(vp), P(vp), ci, ci, ci, sz, P(vp), sz, P(ci), ci]
    L.sgm_match_tiled.argtypes = [vp, vp, vp, ci, ci, sz, vp, sz, ci, ci, P(ci), ci]
    L.sgm_match_tiled_device.argtypes = [vp, vp, vp, ci, ci, sz, vp, sz, ci, ci, P(ci), ci, vp]
    L.sgm_match_tiled_exact.argtypes = [vp, vp, vp, ci, ci, sz, vp, sz, ci, P(ci), ci]
    L.sgm_abi_version.restype = ci
    L.sgm_host_register.argtypes = [vp, vp, sz]
    L.sgm_host_unregister.argtypes = [vp, vp]
    if L.sgm_abi_version() != ABI_VERSION:
        raise ImportError(f"{path}: C-ABI version {L.sgm_abi_version()} != {ABI_VERSION} (include/sgm_hip.h "
                          "SGM_ABI_VERSION): rebuild the library")
    L.sgm_synchronize.argtypes = [vp]
    L.sgm_last_error.argtypes = [vp]
    L.sgm_last_error.restype = ctypes.c_char_p
    L.sgm_set_profiling.argtypes = [vp, ci]
    L.sgm_get_stage_times.argtypes = [vp, P(ctypes.c_float), ci]
    L.sgm_profiled_matches.argtypes = [vp]
    L.sgm_stage_name.argtypes = [vp, ci]
    L.sgm_stage_name.restype = ctypes.c_char_p
    L.sgm_stage_bytes.argtypes = [vp, ci]
    L.sgm_stage_launches.argtypes = [vp, ci]
    L.sgm_disparity_to_msg.argtypes = [vp, vp, sz, ci, ci, ctypes.c_float, ctypes.c_float, vp, sz, vp]
    L.sgm_calc_q.argtypes = [P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_double)]
    L.sgm_calc_q.restype = None
    L.sgm_depth_points.argtypes = [vp, vp, sz, ci, ci, vp, sz, ci, P(ctypes.c_double), ctypes.c_double,
                                   ctypes.c_double, vp, sz, vp, ci, vp, vp]
    L.sgm_stage_bytes.restype = ctypes.c_double
    L.sgm_rectify_map.argtypes = [vp, P(ctypes.c_double), P(ctypes.c_double), ci, P(ctypes.c_double),
                                  P(ctypes.c_double), ci, ci, vp, vp, sz, vp]
    L.sgm_remap_cubic.argtypes = [vp, vp, sz, ci, ci, vp, vp, sz, ci, ci, vp, sz, vp]
    L.sgm_cubic_table.argtypes = [vp]
    L.sgm_set_rectification.argtypes = [vp, vp, vp, vp, vp, sz, ci, ci]
    L.sgm_match_device_batch_rect.argtypes = [vp, P(vp), P(vp), ci, ci, ci, sz, P(vp), P(vp), sz, P(vp), sz, vp]
    L.sgm_cubic_table.restype = None
    L.sgm_debug_census.argtypes = [vp, vp, ci, ci, sz, vp]
    L.sgm_debug_census_path.argtypes = [vp, vp, vp, ci, ci, sz, ci, vp]
    L.sgm_debug_ocv_cost.argtypes = [vp, vp, vp, ci, ci, sz, vp]
    L.sgm_debug_median3.argtypes = [vp, vp, ci, ci]
    L.sgm_debug_speckle.argtypes = [vp, vp, ci, ci, ci, ci, ci]
    L.sgm_debug_path_items.argtypes = [P(SgmParams), ci, ci, ctypes.c_uint, ci, ci, ci, vp, ci]
    _lib = L
    return L


def default_params(mode=MODE_CENSUS8, **kw):
    p = SgmParams()
    load_library().sgm_default_params(ctypes.byref(p), int(mode))
    for k, v in kw.items():
        setattr(p, k, int(v))
    return p


def device_count():
    return int(load_library().sgm_device_count())


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


class SGMError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"sgm status {code}: {msg}")
        self.code = code


def effective_geometry(params, width, height):
    """(minX1, maxX1, width1, D, invalid) — OpenCV computeDisparitySGBM column range."""
    minD, D = params.min_disparity, params.num_disparities
    maxD = minD + D
    minX1 = max(maxD, 0)
    maxX1 = width + min(minD, 0)
    return dict(minX1=minX1, maxX1=maxX1, width1=maxX1 - minX1, D=D, invalid=(minD - 1) * 16)


class Engine:
    """Owning wrapper of one `sgm_handle` (one device, one stream, one workspace)."""

    def __init__(self, device=0, params=None):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.sgm_create(ctypes.byref(h), int(device))
        if rc != SGM_OK:
            raise SGMError(rc, f"cannot open HIP device {device} ({self.lib.sgm_device_count()} visible)")
        self.h = h
        self.device = device
        if params is not None:
            self.set_params(params)

    def close(self):
        if getattr(self, "h", None):
            self.lib.sgm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self):
        e = self.lib.sgm_last_error(self.h)
        return e.decode() if e else ""

    def _check(self, rc):
        if rc != SGM_OK:
            raise SGMError(rc, self.error())

    def set_params(self, p):
        self._check(self.lib.sgm_set_params(self.h, ctypes.byref(p)))

    def get_params(self):
        p = SgmParams()
        self._check(self.lib.sgm_get_params(self.h, ctypes.byref(p)))
        return p

    def match(self, left, right):
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        if left.shape != right.shape or left.ndim != 2:
            raise ValueError("left/right must be equal-size 2-D u8 images")
        h, w = left.shape
        out = np.empty((h, w), np.int16)
        self._check(self.lib.sgm_match(self.h, _ptr(left), _ptr(right), w, h, w, _ptr(out), w))
        return out

    def match_f32(self, left, right, out=None):
        """sgm_match_f32: float32 disparity (x16 fixed point, the CV_32FC1 the node's matcher
        contract returns), converted on the device; `out` (float32 rows) is filled in place."""
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        h, w = left.shape
        if out is None:
            out = np.empty((h, w), np.float32)
        if out.dtype != np.float32 or out.shape != (h, w) or out.strides[1] != 4 or out.strides[0] < 4 * w:
            raise ValueError("out must be a float32 (h, w) row-strided array")
        self._check(self.lib.sgm_match_f32(self.h, _ptr(left), _ptr(right), w, h, w, _ptr(out), out.strides[0] // 4))
        return out

    def match_device(self, d_left, d_right, width, height, stride, d_out, out_stride, stream=None):
        """Device pointers (ints) already resident in HBM; async on `stream` (int handle)."""
        self._check(self.lib.sgm_match_device(self.h, ctypes.c_void_p(d_left), ctypes.c_void_p(d_right), width,
                                              height, stride, ctypes.c_void_p(d_out), out_stride,
                                              ctypes.c_void_p(stream) if stream else None))

    def match_device_batch(self, d_lefts, d_rights, width, height, stride, d_outs, out_stride, stream=None):
        """Frame batch of device pointers; census mode pipelines consecutive frames (the
        aggregation of frame i+1 shares one launch with the WTA of frame i)."""
        n = len(d_lefts)
        arr = ctypes.c_void_p * max(n, 1)
        self._check(self.lib.sgm_match_device_batch(self.h, arr(*d_lefts), arr(*d_rights), n, width, height, stride,
                                                    arr(*d_outs), out_stride,
                                                    ctypes.c_void_p(stream) if stream else None))

    def set_rectification(self, maps_left=None, maps_right=None, map_stride=0, src_width=0, src_height=0):
        """Raw inputs from now on: device matches rectify inside the census through the
        (map_x, map_y) device pointers of each camera (None, None: off)."""
        vp = ctypes.c_void_p
        ml = maps_left or (None, None)
        mr = maps_right or (None, None)
        self._check(self.lib.sgm_set_rectification(self.h, vp(ml[0]), vp(ml[1]), vp(mr[0]), vp(mr[1]), map_stride,
                                                   src_width, src_height))

    def match_device_batch_rect(self, d_lefts, d_rights, width, height, raw_stride, d_rect_lefts, d_rect_rights,
                                rect_stride, d_outs, out_stride, stream=None):
        """match_device_batch on raw frames that also returns the rectified images."""
        n = len(d_lefts)
        arr = ctypes.c_void_p * max(n, 1)
        rl = arr(*d_rect_lefts) if d_rect_lefts is not None else None
        rr = arr(*d_rect_rights) if d_rect_rights is not None else None
        self._check(self.lib.sgm_match_device_batch_rect(self.h, arr(*d_lefts), arr(*d_rights), n, width, height,
                                                         raw_stride, rl, rr, rect_stride, arr(*d_outs), out_stride,
                                                         ctypes.c_void_p(stream) if stream else None))

    def synchronize(self):
        self._check(self.lib.sgm_synchronize(self.h))

    def match_batch(self, lefts, rights, devices=None, outs=None):
        """Host frames, sharded frame i -> devices[i % n] and streamed through pinned rings
        (sgm_match_batch). Row-strided views (one common row stride per side) are passed
        without a copy; `outs` (int16 arrays or row-strided views, one stride) are filled in
        place when given."""
        n = len(lefts)
        h, w = lefts[0].shape

        def rows(arrs, dtype):
            # a row-strided view passes as is; broadcast / overlapping / reversed views
            # (strides[0] < w * itemsize or <= 0) are compacted first
            arrs = [a if (a.dtype == dtype and a.ndim == 2 and a.strides[1] == a.itemsize and
                          a.strides[0] % a.itemsize == 0 and a.strides[0] >= w * a.itemsize)
                    else np.ascontiguousarray(a, dtype) for a in arrs]
            st = {a.strides[0] // a.itemsize for a in arrs}
            if len(st) != 1:   # one stride per side: compact the odd ones out
                arrs = [np.ascontiguousarray(a) for a in arrs]
                st = {w}
            return arrs, st.pop()

        lefts, sl = rows(lefts, np.uint8)
        rights, sr = rows(rights, np.uint8)
        if sl != sr:
            lefts = [np.ascontiguousarray(a) for a in lefts]
            rights = [np.ascontiguousarray(a) for a in rights]
            sl = w
        if outs is None:
            outs = [np.empty((h, w), np.int16) for _ in range(n)]
        so = {a.strides[0] // 2 for a in outs}
        if (len(so) != 1 or any(a.dtype != np.int16 or a.shape != (h, w) or a.strides[1] != 2 for a in outs)):
            raise ValueError("outs must be int16 (h, w) row-strided arrays with one common row stride")
        so = so.pop()
        arr = ctypes.c_void_p * max(n, 1)
        L = arr(*[a.ctypes.data for a in lefts])
        R = arr(*[a.ctypes.data for a in rights])
        O = arr(*[a.ctypes.data for a in outs])
        if devices:
            devs = (ctypes.c_int * len(devices))(*devices)
            nd = len(devices)
        else:
            devs, nd = None, 0
        self._check(self.lib.sgm_match_batch(self.h, L, R, n, w, h, sl, O, so, devs, nd))
        return outs

    def match_tiled(self, left, right, n_bands, halo, devices=None):
        """One frame split into row bands over the devices (overlap mode)."""
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        h, w = left.shape
        out = np.empty((h, w), np.int16)
        if devices:
            devs = (ctypes.c_int * len(devices))(*devices)
            nd = len(devices)
        else:
            devs, nd = None, 0
        self._check(self.lib.sgm_match_tiled(self.h, _ptr(left), _ptr(right), w, h, w, _ptr(out), w, n_bands, halo,
                                             devs, nd))
        return out

    def host_register(self, arr):
        """Page-lock a host array (sgm_host_register): matches into it copy out asynchronously."""
        self._check(self.lib.sgm_host_register(self.h, arr.ctypes.data, arr.nbytes))

    def host_unregister(self, arr):
        self._check(self.lib.sgm_host_unregister(self.h, arr.ctypes.data))

    def match_tiled_device(self, d_left, d_right, width, height, stride, d_out, out_stride, n_bands, halo,
                           devices=None, stream=None):
        """Overlap tile mode on device buffers of this engine's device (C5 frame resident in
        HBM): band b runs on devices[b % len(devices)], rows moved by peer copies."""
        if devices:
            devs = (ctypes.c_int * len(devices))(*devices)
            nd = len(devices)
        else:
            devs, nd = None, 0
        self._check(self.lib.sgm_match_tiled_device(self.h, d_left, d_right, width, height, stride, d_out, out_stride,
                                                    n_bands, halo, devs, nd, stream))

    def match_tiled_exact(self, left, right, n_bands, devices=None):
        """One frame split into row bands over the devices, exact mode: the
        bands' path sweeps continue across the seams through boundary-row exchanges, so the
        result equals match() for any band count."""
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        h, w = left.shape
        out = np.empty((h, w), np.int16)
        if devices:
            devs = (ctypes.c_int * len(devices))(*devices)
            nd = len(devices)
        else:
            devs, nd = None, 0
        self._check(self.lib.sgm_match_tiled_exact(self.h, _ptr(left), _ptr(right), w, h, w, _ptr(out), w, n_bands,
                                                   devs, nd))
        return out

    # -- profiling -------------------------------------------------------------------------
    def set_profiling(self, on=True):
        self._check(self.lib.sgm_set_profiling(self.h, 1 if on else 0))

    def profiled_matches(self):
        return int(self.lib.sgm_profiled_matches(self.h))

    def stage_launches(self):
        """{stage: number of launches recorded since profiling was enabled}"""
        return {self.lib.sgm_stage_name(self.h, i).decode(): int(self.lib.sgm_stage_launches(self.h, i))
                for i in range(len(self.stage_times()))}

    def stage_times(self):
        """[(stage, average ms per launch, algorithmic bytes per launch)], first-launch order"""
        buf = (ctypes.c_float * 16)()
        n = self.lib.sgm_get_stage_times(self.h, buf, 16)
        if n < 0:
            raise SGMError(n, self.error())
        return [(self.lib.sgm_stage_name(self.h, i).decode(), float(buf[i]),
                 float(self.lib.sgm_stage_bytes(self.h, i))) for i in range(n)]

    # -- stage entry points (parity tests) -------------------------------------------------
    # -- after the matcher (device pointers, async on `stream`) ------------------------------
    def disparity_to_msg(self, d_disp, disp_stride, width, height, min_disparity, max_disparity, d_out, out_stride,
                         stream=None):
        """DisparityImage float image from the int16 x16 disparity (generate_disparity.cpp:426-452)."""
        self._check(self.lib.sgm_disparity_to_msg(self.h, ctypes.c_void_p(d_disp), disp_stride, width, height,
                                                  float(min_disparity), float(max_disparity), ctypes.c_void_p(d_out),
                                                  out_stride, ctypes.c_void_p(stream) if stream else None))

    def depth_points(self, d_disp, disp_stride, width, height, q5, depth_min, depth_max, d_color=None,
                     color_stride=0, channels=0, d_depth=None, depth_stride=0, d_points=None, max_points=0,
                     d_num_points=None, stream=None):
        """disparity_to_depth.cpp:127-205; q5 = (Q23, Q03, Q13, Q32, Q33)."""
        q = (ctypes.c_double * 5)(*[float(v) for v in q5])
        vp = ctypes.c_void_p
        self._check(self.lib.sgm_depth_points(self.h, vp(d_disp), disp_stride, width, height, vp(d_color),
                                              color_stride, channels, q, float(depth_min), float(depth_max),
                                              vp(d_depth), depth_stride, vp(d_points), max_points,
                                              vp(d_num_points), vp(stream) if stream else None))

    def rectify_map(self, K, D, R, P, width, height, d_map_x, d_map_y, map_stride, stream=None):
        """initUndistortRectifyMap(K, D, R, P, (width, height), CV_32FC1) into device float maps
        (generate_disparity.cpp:379-380). R None = identity; D: 0/4/5/8/12 coefficients."""
        dv = ctypes.c_double
        k = (dv * 9)(*np.asarray(K, np.float64).ravel())
        dd = np.asarray([] if D is None else D, np.float64).ravel()
        darr = (dv * max(len(dd), 1))(*dd)
        r = (dv * 9)(*np.asarray(R, np.float64).ravel()) if R is not None else None
        pp = (dv * 12)(*np.asarray(P, np.float64).ravel())
        vp = ctypes.c_void_p
        self._check(self.lib.sgm_rectify_map(self.h, k, darr, len(dd), r, pp, width, height, vp(d_map_x),
                                             vp(d_map_y), map_stride, vp(stream) if stream else None))

    def remap_cubic(self, d_src, src_stride, src_w, src_h, d_map_x, d_map_y, map_stride, width, height, d_dst,
                    dst_stride, stream=None):
        """cv::remap(src, dst, map_x, map_y, INTER_CUBIC, BORDER_CONSTANT) on device buffers
        (generate_disparity.cpp:383)."""
        vp = ctypes.c_void_p
        self._check(self.lib.sgm_remap_cubic(self.h, vp(d_src), src_stride, src_w, src_h, vp(d_map_x), vp(d_map_y),
                                             map_stride, width, height, vp(d_dst), dst_stride,
                                             vp(stream) if stream else None))

    def census(self, img):
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        out = np.empty((h, w), np.uint64)
        self._check(self.lib.sgm_debug_census(self.h, _ptr(img), w, h, w, _ptr(out)))
        return out

    def census_path(self, left, right, direction):
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        h, w = left.shape
        e = effective_geometry(self.get_params(), w, h)
        vol = np.zeros((h, max(e["width1"], 0), e["D"]), np.uint8)
        self._check(self.lib.sgm_debug_census_path(self.h, _ptr(left), _ptr(right), w, h, w, int(direction),
                                                   _ptr(vol)))
        return vol

    def ocv_cost(self, left, right):
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        h, w = left.shape
        e = effective_geometry(self.get_params(), w, h)
        C = np.zeros((h, max(e["width1"], 0), e["D"]), np.int16)
        self._check(self.lib.sgm_debug_ocv_cost(self.h, _ptr(left), _ptr(right), w, h, w, _ptr(C)))
        return C

    def median3(self, disp):
        d = np.ascontiguousarray(disp, np.int16).copy()
        h, w = d.shape
        self._check(self.lib.sgm_debug_median3(self.h, _ptr(d), w, h))
        return d

    def filter_speckles(self, disp, new_val, max_size, max_diff):
        d = np.ascontiguousarray(disp, np.int16).copy()
        h, w = d.shape
        self._check(self.lib.sgm_debug_speckle(self.h, _ptr(d), w, h, new_val, max_size, max_diff))
        return d


def calc_q(K, P_right, P_left):
    """calc_q (disparity_to_depth.cpp:62-84) through the C-ABI: 4x4 float64 Q."""
    lib = load_library()
    dv = ctypes.c_double
    k = (dv * 9)(*np.asarray(K, np.float64).ravel())
    pr = (dv * 12)(*np.asarray(P_right, np.float64).ravel())
    pl = (dv * 12)(*np.asarray(P_left, np.float64).ravel())
    q = (dv * 16)()
    lib.sgm_calc_q(k, pr, pl, q)
    return np.array(q[:], np.float64).reshape(4, 4)


def _side_stream(torch):
    """A stream ordered after everything already queued on torch's current stream (the
    library's NULL-stream argument means the handle's own stream, not torch's)."""
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    return st


def cubic_table():
    """The INTER_CUBIC int16 weight table of the library (host code, no device needed)."""
    lib = load_library()
    t = np.empty((1024, 16), np.int16)
    lib.sgm_cubic_table(t.ctypes.data_as(ctypes.c_void_p))
    return t


def rectify(engine, image, K, D, R, P, maps=None):
    """The node's rectify(image, camera_info) (generate_disparity.cpp:370-386) on the GPU:
    initUndistortRectifyMap + remap INTER_CUBIC / BORDER_CONSTANT. `maps` (map_x, map_y
    device tensors from a previous call) skips the map computation — the map depends only
    on the calibration. Returns (rectified u8 image as numpy, maps)."""
    import torch
    img = torch.as_tensor(np.ascontiguousarray(image, np.uint8)).cuda()
    h, w = img.shape
    if maps is None:
        mx = torch.empty((h, w), dtype=torch.float32, device="cuda")
        my = torch.empty((h, w), dtype=torch.float32, device="cuda")
        maps = (mx, my)
    out = torch.empty((h, w), dtype=torch.uint8, device="cuda")
    stream = _side_stream(torch)
    if len(maps) == 2:
        engine.rectify_map(K, D, R, P, w, h, maps[0].data_ptr(), maps[1].data_ptr(), w, stream.cuda_stream)
        maps = (maps[0], maps[1], True)
    engine.remap_cubic(img.data_ptr(), w, w, h, maps[0].data_ptr(), maps[1].data_ptr(), w, w, h, out.data_ptr(), w,
                       stream.cuda_stream)
    stream.synchronize()
    return out.cpu().numpy(), maps


def q_terms(Q):
    """The five Q entries the depth node uses (disparity_to_depth.cpp:134-138)."""
    Q = np.asarray(Q, np.float64)
    return (Q[2, 3], Q[0, 3], Q[1, 3], Q[3, 2], Q[3, 3])


def disp_info_to_depth(engine, disp_image, color, Q, depth_min=0.0, depth_max=100.0, gen_point_cloud=True):
    """dispInfoMsg2depthMsg (disparity_to_depth.cpp:94-218) on the GPU: the DisparityImage
    float image (+ MONO8/BGR8 color) -> (depth float32 HxW, points Nx3 float32, rgba N)."""
    import torch
    d = torch.as_tensor(np.ascontiguousarray(disp_image, np.float32)).cuda()
    h, w = d.shape
    c = None
    ch = 0
    if color is not None:
        c = torch.as_tensor(np.ascontiguousarray(color, np.uint8)).cuda()
        ch = 1 if c.dim() == 2 else 3
    depth = torch.empty((h, w), dtype=torch.float32, device="cuda")
    pts = torch.empty((h * w if gen_point_cloud else 1, 4), dtype=torch.float32, device="cuda")
    n = torch.zeros(1, dtype=torch.int32, device="cuda")
    stream = _side_stream(torch)
    engine.depth_points(d.data_ptr(), w, w, h, q_terms(Q), depth_min, depth_max,
                        c.data_ptr() if c is not None else None, w * ch, ch, depth.data_ptr(), w,
                        pts.data_ptr() if gen_point_cloud else None, h * w if gen_point_cloud else 0,
                        n.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    k = int(n.item())
    p = pts[:k].cpu().numpy() if gen_point_cloud else np.zeros((0, 4), np.float32)
    return depth.cpu().numpy(), p[:, :3].copy(), p[:, 3].copy().view(np.uint32)


def right_matcher_params(p):
    """cv::ximgproc::createRightMatcher for a StereoSGBM: minD' = -(minD + D) + 1, same D /
    block / P1 / P2 / mode / preFilterCap, uniqueness 0, disp12MaxDiff 1e6, no speckle filter
    (reference calls it at matcherOpenCVSGBM.cpp:48)."""
    return p.copy(min_disparity=-(p.min_disparity + p.num_disparities) + 1, uniqueness_ratio=0,
                  disp12_max_diff=1000000, speckle_window_size=0)


class MatcherHIPSGM:
    """`MatcherHIPSGM : AbstractStereoMatcher` host mirror.

    Same method names, argument meaning and error behaviour as the reference's
    MatcherOpenCVSGBM (matcherOpenCVSGBM.{h,cpp}); compute delegated to libsgm_hip.so.
    `mode` picks the engine mode (the reference's SGBM path never sets a mode, Q1, so the
    OpenCV-compatible default is MODE_SGBM = 5 directions; env SGM_HIP_MODE overrides).
    """

    def __init__(self, param_file=" ", image_size=(0, 0), device=0, mode=None):
        self.param_file = param_file
        self.image_size = (0, 0)          # Q5: the base ctor ignores _image_size
        self.downsample_scale = 1.0
        self.min_disparity = 0
        self.disparity_range = 64
        self.window_size = 9
        self.interpolate = False
        self.left = None
        self.right = None
        self.disparity_lr = None
        self.disparity_rl = None
        if mode is None:
            mode = int(os.environ.get("SGM_HIP_MODE", MODE_OCV_SGBM5))
        self.device = device
        self.mode = mode
        self.init()

    # --- AbstractStereoMatcher ----------------------------------------------------------
    def init(self):
        # cv::StereoSGBM::create(64, 9, 5) equivalent starting point (matcherOpenCVSGBM.cpp:14)
        p = default_params(self.mode)
        p.ocv_compat = ocv_compat_from_env(p.ocv_compat)
        p.min_disparity, p.num_disparities, p.block_size = 64, 9, 5
        p.p1 = p.p2 = p.uniqueness_ratio = p.disp12_max_diff = p.prefilter_cap = 0
        p.speckle_window_size = p.speckle_range = 0
        self.params = p
        self._engine = None               # opened lazily at the first match (Q5 / §8b)

    def setImages(self, left, right):
        if left.shape != right.shape:
            sys.stderr.write("Images MUST be the same resolution\n")
            return
        # scale 1 (the node always passes 1): cv::resize short-circuits to a copy
        self.left = np.array(left, copy=True)
        self.right = np.array(right, copy=True)
        self.image_size = (self.left.shape[1], self.left.shape[0])

    def setDownsampleScale(self, scale=1.0):
        self.downsample_scale = scale

    def setDisparityRange(self, disparity_range):
        if disparity_range <= 0:
            disparity_range = ((self.image_size[0] // 8) + 15) & -16
        self.disparity_range = disparity_range
        self.params.num_disparities = int(disparity_range)

    def setWindowSize(self, window_size):
        self.window_size = window_size
        self.params.block_size = int(window_size)

    def setInterpolation(self, enable):
        self.interpolate = bool(enable)

    def setMinDisparity(self, min_disparity):
        self.min_disparity = min_disparity
        self.params.min_disparity = int(min_disparity)

    def setUniquenessRatio(self, ratio):
        self.params.uniqueness_ratio = int(ratio)          # Q7: double in cfg -> int

    def setSpeckleFilterWindow(self, window):
        self.params.speckle_window_size = int(window)

    def setSpeckleFilterRange(self, rng):
        self.params.speckle_range = int(rng)

    def setDisp12MaxDiff(self, diff):
        self.params.disp12_max_diff = int(diff)

    def setPreFilterCap(self, cap):
        self.params.prefilter_cap = int(cap)

    def setP1(self, p1):
        self.params.p1 = int(p1)                           # OpenCV setP1(int): truncation

    def setP2(self, p2):
        self.params.p2 = int(p2)

    def setTextureThreshold(self, threshold):              # not used by SGBM
        pass

    def setPreFilterSize(self, size):                      # not used by SGBM
        pass

    def setOcclusionDetection(self, enable):               # not used by SGBM
        pass

    def _engine_for(self):
        if self._engine is None:
            self._engine = Engine(self.device)
        return self._engine

    def _run(self, params, a, b, f32=False):
        eng = self._engine_for()
        eng.set_params(params)
        return eng.match_f32(a, b) if f32 else eng.match(a, b)

    def forwardMatch(self):
        try:
            if self.interpolate:
                # Q3: the WLS output is discarded and disparity_rl (CV_16S) replaces disparity_lr
                self.backwardMatch()
                self.disparity_lr = self.disparity_rl.astype(np.float32)
            else:
                # CV_32FC1 converted on the device (sgm_match_f32)
                self.disparity_lr = self._run(self.params, self.left, self.right, f32=True)
            return 0
        except Exception as e:  # mirrors the catch(cv::Exception&) -> -1
            sys.stderr.write("Error in HIP SGM parameters\n%s\n" % e)
            return -1

    def backwardMatch(self):
        self.disparity_rl = self._run(right_matcher_params(self.params), self.right, self.left)
        return 0

    def match(self):
        code = self.forwardMatch()
        if code == 0:
            self.disparity_lr = self.disparity_lr.astype(np.float32)
        return code

    def getDisparity(self):
        return None if self.disparity_lr is None else self.disparity_lr.copy()

    def getBackDisparity(self):
        return None if self.disparity_rl is None else self.disparity_rl.copy()

    def getLeftImage(self):
        return self.left

    def getRighttImage(self):  # (sic) reference spelling, abstractStereoMatcher.h:71
        return self.right


# ---------------------------------------------------------------- node-level plumbing
NODE_DEFAULTS = dict(stereo_algorithm=CV_StereoBM, min_disparity=9, disparity_range=64,
                     correlation_window_size=15, uniqueness_ratio=15, texture_threshold=10,
                     speckle_size=100, speckle_range=4, disp12MaxDiff=0, p1=200.0, p2=400.0,
                     interp=False, prefilter_cap=31, prefilter_size=9)  # generate_disparity.cpp:90-112


def update_matcher(matcher, cfg):
    """updateMatcher() — generate_disparity.cpp:241-261 (disp12MaxDiff is NOT forwarded, Q1)."""
    matcher.setDisparityRange(cfg["disparity_range"])
    matcher.setWindowSize(cfg["correlation_window_size"])
    matcher.setMinDisparity(cfg["min_disparity"])
    matcher.setUniquenessRatio(int(cfg["uniqueness_ratio"]))
    matcher.setSpeckleFilterRange(cfg["speckle_range"])
    matcher.setSpeckleFilterWindow(cfg["speckle_size"])
    matcher.setPreFilterCap(cfg["prefilter_cap"])
    matcher.setP1(cfg["p1"])
    matcher.setP2(cfg["p2"])
    matcher.setTextureThreshold(cfg["texture_threshold"])
    matcher.setPreFilterSize(cfg["prefilter_size"])
    matcher.setInterpolation(cfg["interp"])


def parameter_callback(config, state):
    """parameterCallback() sanitising (generate_disparity.cpp:735-845) for the HIP entry.

    `state` holds `first` (bool) and the node globals; returns the (possibly rewritten)
    config like dynamic_reconfigure does."""
    config = dict(config)
    if state.get("first", True):
        for k in NODE_DEFAULTS:
            config[k] = state.get(k, NODE_DEFAULTS[k])
        state["first"] = False
        return config
    config["prefilter_size"] |= 1
    if config["stereo_algorithm"] in (CV_StereoBM, CV_StereoSGBM, CV_StereoBMCuda, CV_StereoBPCuda,
                                      CV_StereoCSBPCuda, HIP_StereoSGM):
        config["correlation_window_size"] |= 1
        config["disparity_range"] = (config["disparity_range"] // 16) * 16
    if config["stereo_algorithm"] == I3DR_StereoSGM and config["correlation_window_size"] > 17:
        config["correlation_window_size"] = 17
    for k in NODE_DEFAULTS:
        state[k] = config[k]
    return config


def bgr2gray(img):
    """cv::cvtColor(COLOR_BGR2GRAY) for 8U: fixed-point 14-bit coefficients, round half up."""
    img = np.asarray(img)
    if img.ndim == 2:
        return img.astype(np.uint8, copy=True)
    b, g, r = (img[..., i].astype(np.int32) for i in range(3))
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


def stereo_match(matcher, left_mono, right_mono):
    """stereo_match() — generate_disparity.cpp:334-368: empty result on failure."""
    matcher.setDownsampleScale(1)
    matcher.setImages(left_mono, right_mono)
    code = matcher.match()
    if code == 0:
        return matcher.getDisparity()
    sys.stderr.write(f"Exit code:{code}\nFailed to compute stereo match\nPlease check parameters are valid.\n")
    return np.empty((0, 0), np.float32)


def process_disparity(matcher, left_rect, right_rect, f, T, depth_min=0.0, depth_max=10.0):
    """processDisparity() — generate_disparity.cpp:398-456. Returns the DisparityImage fields
    or None when the match failed (the node returns -1 and publishes nothing)."""
    disp = stereo_match(matcher, bgr2gray(left_rect), bgr2gray(right_rect))
    if disp.size == 0:
        return None
    dmat = (disp.astype(np.float32) * np.float32(1.0 / 16)).astype(np.float32)
    min_disp = np.float32(T * f / depth_max)
    with np.errstate(divide="ignore"):
        max_disp = np.float32(T * f / depth_min) if depth_min != 0 else np.float32(np.inf)  # Q8
    dmat[dmat < min_disp] = MISSING_Z
    dmat[dmat > max_disp] = MISSING_Z
    return dict(image=dmat, f=f, T=T, min_disparity=float(min_disp), max_disparity=float(max_disp),
                delta_d=1.0 / 16, height=dmat.shape[0], width=dmat.shape[1], encoding="32FC1",
                step=dmat.shape[1] * 4)
