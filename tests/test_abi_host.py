"""CPU tests of the C-ABI library surface and the host-side mirror (no compute calls)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sgm_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sgm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_full_abi():
    syms = declared_symbols()
    for s in ("sgm_create", "sgm_destroy", "sgm_set_params", "sgm_match", "sgm_match_device",
              "sgm_match_batch", "sgm_last_error", "sgm_device_count"):
        assert s in syms


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (sgm_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, f"declared but not exported: {missing}"
    for s in declared_symbols():
        assert hasattr(lib, s)
    assert sorted(pkg.EXPORTS) == declared_symbols()


def test_library_is_gfx950_code_object(pkg):
    blob = open(pkg.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob          # embedded gfx950 code object


def test_default_params_match_node_defaults(pkg):
    p = pkg.default_params(pkg.MODE_OCV_SGBM5)
    # generate_disparity.cpp:100-112
    assert (p.min_disparity, p.num_disparities, p.block_size, p.p1, p.p2, p.uniqueness_ratio,
            p.speckle_window_size, p.speckle_range, p.prefilter_cap) == (9, 64, 15, 200, 400, 15, 100, 4, 31)
    c = pkg.default_params(pkg.MODE_CENSUS8)
    assert (c.p1, c.p2, c.uniqueness_ratio, c.subpixel, c.lr_check) == (10, 120, 5, 1, 1)
    # the OpenCV build the OCV modes reproduce: melodic (the reference's Dockerfile:1), census: n/a
    assert p.ocv_compat == pkg.COMPAT_MELODIC == 7 and c.ocv_compat == 0
    assert ctypes.sizeof(pkg.SgmParams) == 15 * 4


@pytest.mark.parametrize("val,bits", [(None, 7), ("melodic", 7), ("noetic", 2), ("scalar", 0), ("5", 5),
                                      ("0x3", 3), ("Melodic", 7), (" melodic ", 7), ("NOETIC\t", 2), ("", 7),
                                      ("melodik", 7), ("3x", 7), ("  ", 7)])
def test_ocv_compat_env(pkg, monkeypatch, val, bits):
    """SGM_HIP_OCV_COMPAT selects the OpenCV build, in the Python mirror's
    MatcherHIPSGM and in the C++ adapter core alike: case and blanks ignored, an unparseable
    value warns and keeps the melodic default."""
    if val is None:
        monkeypatch.delenv("SGM_HIP_OCV_COMPAT", raising=False)
    else:
        monkeypatch.setenv("SGM_HIP_OCV_COMPAT", val)
    assert pkg.ocv_compat_from_env() == bits
    assert pkg.MatcherHIPSGM(" ", (0, 0), mode=pkg.MODE_OCV_SGBM5).params.ocv_compat == bits
    exe = os.path.join(ROOT, "i3dr_stereo_camera-ros_amd", "lib", "plugin_core_test")
    r = subprocess.run([exe, "compat"], capture_output=True, text=True)
    assert r.returncode == 0 and int(r.stdout) == bits, r.stderr


@pytest.mark.parametrize("mode,D,expect", [("census", 64, 0), ("census", 24, -2), ("census", 0, -2),
                                           ("census", 528, -5), ("census", 512, 0),
                                           ("ocv", 528, 0), ("ocv", 2048, 0), ("ocv", 2064, -5), ("ocv", 40, -2)])
def test_check_params(pkg, mode, D, expect):
    """D limits: census 512 (u8 path engine); the OpenCV modes 2048, the top of the node's
    cfg range (cfg/i3DR_Disparity.cfg:27, disparity_range <= 2056 rounded down to x16)."""
    lib = pkg.load_library()
    p = pkg.default_params(pkg.MODE_CENSUS8 if mode == "census" else pkg.MODE_OCV_SGBM5, num_disparities=D)
    assert lib.sgm_check_params(ctypes.byref(p), 640, 480) == expect


def test_no_device_fails_loudly(pkg):
    """Without a GPU the product path must fail, never fall back to a CPU implementation."""
    if pkg.device_count() > 0:
        pytest.skip("a HIP device is visible")
    lib = pkg.load_library()
    h = ctypes.c_void_p()
    assert lib.sgm_create(ctypes.byref(h), 0) == pkg.SGM_ERR_DEVICE
    with pytest.raises(pkg.SGMError):
        pkg.Engine(0)
    m = pkg.MatcherHIPSGM(" ", (64, 48))
    z = np.zeros((48, 64), np.uint8)
    m.setImages(z, z)
    assert m.match() == -1        # the reference's forwardMatch error code


def test_matcher_setter_semantics(pkg):
    m = pkg.MatcherHIPSGM(" ", (640, 480), mode=pkg.MODE_OCV_SGBM5)
    assert (m.params.min_disparity, m.params.num_disparities, m.params.block_size) == (64, 9, 5)  # create(64,9,5)
    m.setDisparityRange(0)                       # image_size not set yet (Q5): ((0/8)+15)&-16
    assert m.params.num_disparities == 0
    z = np.zeros((480, 640), np.uint8)
    m.setImages(z, z)
    m.setDisparityRange(-1)
    assert m.params.num_disparities == ((640 // 8) + 15) & -16
    m.setP1(200.7)
    m.setP2(399.9)
    assert (m.params.p1, m.params.p2) == (200, 399)
    m.setUniquenessRatio(15.8)
    assert m.params.uniqueness_ratio == 15
    m.setTextureThreshold(5)
    m.setPreFilterSize(9)
    m.setOcclusionDetection(True)               # no-ops


def test_right_matcher_params(pkg):
    p = pkg.default_params(pkg.MODE_OCV_SGBM5, min_disparity=9, num_disparities=64)
    r = pkg.right_matcher_params(p)
    assert (r.min_disparity, r.num_disparities, r.uniqueness_ratio, r.disp12_max_diff, r.speckle_window_size) == \
        (-72, 64, 0, 1000000, 0)


def test_parameter_callback_sanitises(pkg):
    state = {"first": True}
    cfg = pkg.parameter_callback({}, state)           # first call pushes node values into config
    assert cfg["min_disparity"] == 9 and not state["first"]
    cfg.update(stereo_algorithm=pkg.HIP_StereoSGM, correlation_window_size=10, disparity_range=70,
               prefilter_size=8)
    cfg = pkg.parameter_callback(cfg, state)
    assert cfg["correlation_window_size"] == 11 and cfg["disparity_range"] == 64 and cfg["prefilter_size"] == 9
    cfg.update(stereo_algorithm=pkg.I3DR_StereoSGM, correlation_window_size=31)
    assert pkg.parameter_callback(cfg, state)["correlation_window_size"] == 17


def test_bgr2gray_fixed_point(pkg):
    img = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [10, 200, 30]]], np.uint8)
    g = pkg.bgr2gray(img)
    exp = [(b * 1868 + gg * 9617 + r * 4899 + 8192) >> 14 for b, gg, r in img[0].astype(int)]
    assert g[0].tolist() == exp


class _StubMatcher:
    """Stand-in with the plugin interface, returning a fixed x16 disparity."""

    def __init__(self, disp, code=0):
        self.disp, self.code = disp, code

    def setDownsampleScale(self, s):
        pass

    def setImages(self, a, b):
        self.shape = a.shape

    def match(self):
        return self.code

    def getDisparity(self):
        return self.disp.astype(np.float32)


def test_process_disparity_plumbing(pkg):
    disp = np.array([[-16, 0, 16 * 3, 16 * 40], [16 * 100, 8, 24, 160]], np.int16)
    z = np.zeros((2, 4), np.uint8)
    out = pkg.process_disparity(_StubMatcher(disp), z, z, f=500.0, T=0.1, depth_min=0.5, depth_max=10.0)
    img = out["image"]
    assert img.dtype == np.float32 and out["delta_d"] == 1 / 16
    assert out["min_disparity"] == pytest.approx(5.0) and out["max_disparity"] == pytest.approx(100.0)
    exp = disp / 16.0
    exp[(exp < 5.0) | (exp > 100.0)] = pkg.MISSING_Z
    assert np.array_equal(img, exp.astype(np.float32))
    assert pkg.process_disparity(_StubMatcher(disp, code=-1), z, z, 500.0, 0.1) is None


def test_plugin_core_cpp_setters():
    exe = os.path.join(ROOT, "i3dr_stereo_camera-ros_amd", "lib", "plugin_core_test")
    r = subprocess.run([exe, "setters"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
