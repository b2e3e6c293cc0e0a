"""GPU parity — OpenCV-StereoSGBM-compatible modes (the reference's actual CPU path).

Bit-exact against the oracle's raster restatement of cv::StereoSGBM (MODE_SGBM = the
reference's default, MODE_HH = cfg `fullDP`), including the aggregated cost volume C',
the node defaults (C1: 640x480, minD 9, D 64, block 15) and the plugin-level paths.
"""
import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("h,w,minD,D,block,cap", [(12, 50, 0, 16, 5, 31), (9, 45, 4, 16, 7, 15),
                                                  (4, 40, -3, 16, 9, 63), (17, 70, 2, 32, 3, 1),
                                                  (40, 200, 9, 64, 15, 31), (30, 300, 0, 128, 11, 20),
                                                  (130, 333, 5, 48, 9, 31),       # 3 vsum row segments
                                                  (70, 400, 0, 256, 101, 31)])    # LDS tile too big: unfused
def test_ocv_cost_volume(engine, oracle, pkg, mode, h, w, minD, D, block, cap):
    rng = np.random.default_rng(h * w + mode)
    left = rng.integers(0, 256, (h, w), dtype=np.uint8)
    right = rng.integers(0, 256, (h, w), dtype=np.uint8)
    p = pkg.default_params(mode, min_disparity=minD, num_disparities=D, block_size=block, prefilter_cap=cap,
                           p1=8, p2=32)
    engine.set_params(p)
    got = engine.ocv_cost(left, right)
    ref = oracle.ocv_cost(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} cost cells differ"


OCV_CASES = [
    (0, dict()),                                                     # node defaults
    (1, dict()),
    (0, dict(min_disparity=0, num_disparities=32, block_size=5, speckle_window_size=0)),
    (1, dict(min_disparity=-6, num_disparities=48, block_size=3, p1=8, p2=60)),
    (0, dict(min_disparity=2, num_disparities=128, block_size=9, uniqueness_ratio=5, disp12_max_diff=2)),
    (1, dict(min_disparity=0, num_disparities=16, block_size=1, prefilter_cap=63, speckle_range=1)),
    (0, dict(min_disparity=0, num_disparities=256, block_size=7)),
]


@pytest.mark.parametrize("mode,kw", OCV_CASES, ids=[str(i) for i in range(len(OCV_CASES))])
def test_ocv_pipeline(engine, oracle, synth, pkg, mode, kw):
    p = pkg.default_params(mode, **kw)
    D, minD = p.num_disparities, p.min_disparity
    h, w = 57, max(D + minD, 0) + 120
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=D + mode)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("mode", [0, 1])
def test_ocv_node_defaults_c1(engine, oracle, synth, pkg, mode):
    """BASELINE config C1 geometry: 640x480, generate_disparity node defaults."""
    left, right, _ = synth.stereo_pair(480, 640, 9, 64, seed=1)
    p = pkg.default_params(mode)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


COMPATS = pytest.mark.parametrize("compat", [0, 7], ids=["scalar", "melodic"])   # sgm_params.ocv_compat


@COMPATS
@pytest.mark.parametrize("nobuf", ["", "1"], ids=["buf32", "ptr64"])
@pytest.mark.parametrize("lanes", ["16", "32"])
@pytest.mark.parametrize("mode,h,w,minD,D,block", [(0, 480, 640, 9, 64, 15), (1, 96, 500, 0, 128, 5),
                                                   (0, 40, 600, -4, 256, 7), (1, 33, 200, 3, 48, 3),
                                                   (1, 24, 640, -3, 480, 9), (0, 20, 700, 147, 400, 21)])
def test_ocv_path_lanes_per_line(engine, oracle, synth, pkg, monkeypatch, nobuf, lanes, mode, h, w, minD, D, block,
                                 compat):
    """Both path-kernel shapes (16 and 32 lanes per line, SGM_OCV_LPL) and both addressing
    schemes (32-bit buffer offsets; the 64-bit clamped pointers of > 2 GB volumes,
    SGM_OCV_NO_BUF) on the same inputs."""
    monkeypatch.setenv("SGM_OCV_LPL", lanes)
    if nobuf:
        monkeypatch.setenv("SGM_OCV_NO_BUF", nobuf)
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=h + D)
    p = pkg.default_params(mode, min_disparity=minD, num_disparities=D, block_size=block, ocv_compat=compat)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("uniq", [0, 10])
def test_ocv_saturated_sums(engine, oracle, pkg, mode, uniq):
    """Noise under a 21x21 box and a large P2 saturates S at MAX_COST for every d of some
    pixels: OpenCV's strict `Sval < minS` from minS = MAX_COST then leaves bestDisp = -1, so
    the pixel is INVALID whatever the uniqueness ratio (found by tests/test_gpu_fuzz.py)."""
    rng = np.random.default_rng(56 + mode)
    left = rng.integers(0, 256, (24, 200), dtype=np.uint8)
    right = rng.integers(0, 256, (24, 200), dtype=np.uint8)
    p = pkg.default_params(mode, min_disparity=-3, num_disparities=128, block_size=21, p1=128, p2=912,
                           uniqueness_ratio=uniq, prefilter_cap=27, speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@COMPATS
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("force", ["", "1"], ids=["auto", "forced"])
def test_ocv_wide_path_costs(engine, oracle, synth, pkg, monkeypatch, mode, force, compat):
    """Boxes whose sums can wrap int16 (21x21, preFilterCap 62): OpenCV's CostType cost
    volume wraps, a path cost can leave int16, and S adds the int values — the engine keeps
    int32 path volumes there (Geom::wide, automatic from the parameters); the SIMD builds
    (melodic) saturate instead: the sequential saturating cost + int16 saturating paths.
    `forced` runs an ordinary configuration through those kernels too (SGM_OCV_WIDE=1)."""
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


@pytest.mark.parametrize("seed", [3791, 4079, 4568])
def test_ocv_negative_min_cost_disp2(engine, oracle, synth, pkg, seed):
    """Fuzz cases (tests/test_gpu_fuzz.py seeds) where wrapped costs make a pixel's minS
    negative: disp2's "cost > minS" update must compare signed CostType values."""
    from test_gpu_fuzz import _case, _images
    rng, mode, h, w, kw, kind = _case(pkg, seed)
    p = pkg.default_params(mode, **kw)
    engine.set_params(p)
    left, right = _images(rng, synth, h, w, kw["min_disparity"], kw["num_disparities"], kind, seed)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


def test_ocv_small_images_bottom_rows(engine, oracle, pkg):
    """Heights below the SAD window (every row hits OpenCV's no-recompute rule)."""
    rng = np.random.default_rng(7)
    for mode in (0, 1):
        for h in (1, 2, 5, 8):
            left = rng.integers(0, 256, (h, 80), dtype=np.uint8)
            right = rng.integers(0, 256, (h, 80), dtype=np.uint8)
            p = pkg.default_params(mode, min_disparity=0, num_disparities=16, block_size=15)
            engine.set_params(p)
            assert np.array_equal(engine.match(left, right), oracle.match(to_oracle_params(oracle, p), left, right))


def test_matcher_plugin_mirror(pkg, oracle, synth):
    """MatcherHIPSGM + process_disparity exactly as the node drives them (updateMatcher)."""
    left, right, _ = synth.stereo_pair(120, 320, 9, 64, seed=5)
    m = pkg.MatcherHIPSGM(" ", (320, 120), mode=pkg.MODE_OCV_SGBM5)
    m.setImages(left, right)
    pkg.update_matcher(m, pkg.NODE_DEFAULTS)
    assert m.match() == 0
    ref = oracle.match(oracle.make_params(0), left, right).astype(np.float32)
    assert np.array_equal(m.getDisparity(), ref)
    out = pkg.process_disparity(m, left, right, f=700.0, T=0.12, depth_min=0.3, depth_max=20.0)
    exp = ref / 16.0
    exp[(exp < np.float32(0.12 * 700.0 / 20.0)) | (exp > np.float32(0.12 * 700.0 / 0.3))] = pkg.MISSING_Z
    assert np.allclose(out["image"], exp, rtol=0, atol=0)


def test_matcher_interp_returns_right_view(pkg, oracle, synth):
    """interp=true: the reference returns the right matcher's disparity (Q3)."""
    left, right, _ = synth.stereo_pair(80, 240, 0, 48, seed=6)
    m = pkg.MatcherHIPSGM(" ", (240, 80), mode=pkg.MODE_OCV_SGBM5)
    m.setImages(left, right)
    cfg = dict(pkg.NODE_DEFAULTS, min_disparity=0, disparity_range=48, interp=True)
    pkg.update_matcher(m, cfg)
    assert m.match() == 0
    rp = pkg.right_matcher_params(m.params)
    ref = oracle.match(to_oracle_params(oracle, rp), right, left).astype(np.float32)
    assert np.array_equal(m.getDisparity(), ref)
    assert (ref[ref != (rp.min_disparity - 1) * 16] <= 0).mean() > 0.9   # right-view disparities are <= 0


def test_plugin_core_cpp_init_and_match(tmp_path, oracle, synth):
    """C++ host adapter core: the init_stereo_matchers warm-up + a node-default match."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "i3dr_stereo_camera-ros_amd",
                       "lib", "plugin_core_test")
    r = subprocess.run([exe, "init"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    left, right, _ = synth.stereo_pair(96, 256, 9, 64, seed=8)
    lp, rp, op = tmp_path / "l.raw", tmp_path / "r.raw", tmp_path / "o.f32"
    left.tofile(lp)
    right.tofile(rp)
    r = subprocess.run([exe, "match", str(lp), str(rp), "256", "96", str(op), "0", "64", "9", "0"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(op, np.float32).reshape(96, 256)
    assert np.array_equal(got, oracle.match(oracle.make_params(0), left, right).astype(np.float32))


@COMPATS
@pytest.mark.parametrize("wide", ["", "1"], ids=["plain", "flagged"])
@pytest.mark.parametrize("mode,h,w,minD,D,block,spk", [(0, 20, 1400, 0, 1024, 5, 100), (1, 24, 1300, -7, 784, 3, 0),
                                                       (0, 12, 2300, 3, 2048, 7, 0), (1, 28, 2200, 0, 1536, 5, 0),
                                                       (0, 16, 1340, -1, 1296, 3, 10), (1, 20, 1200, 0, 1040, 5, 0)])
def test_ocv_large_disparity_ranges(engine, oracle, synth, pkg, monkeypatch, wide, mode, h, w, minD, D, block, spk,
                                    compat):
    """D > 512 in the OpenCV modes (the node's cfg allows disparity ranges up to 2048):
    64-lane path lines (16 or 32 values per lane; D % 32 = 16 above 1024 leaves one lane
    straddling D, found by the D > 512 fuzz) and the one-pixel-per-wave WTA in chunks of 1024
    disparities, int16 and int32 (SGM_OCV_WIDE) volumes."""
    if wide:
        monkeypatch.setenv("SGM_OCV_WIDE", wide)
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), min(D, 256), seed=D + h)
    p = pkg.default_params(mode, min_disparity=minD, num_disparities=D, block_size=block, speckle_window_size=spk,
                           ocv_compat=compat)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
    assert (ref[:, max(minD + D, 0):] != (minD - 1) * 16).any()      # some matched pixels to compare


@pytest.mark.parametrize("block", [61, 63, 65, 131])
def test_ocv_tall_boxes(engine, oracle, synth, pkg, block):
    """Tall SAD boxes (the cfg allows windows up to 255): the fused pixel-cost + box kernel
    up to its 64 KB tile, the unfused pixcost + hsum pair beyond it, long vertical windows."""
    left, right, _ = synth.stereo_pair(150, 320, 0, 32, seed=block)
    p = pkg.default_params(0, min_disparity=0, num_disparities=32, block_size=block, speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("streams", ["3", "1", "8"])
@pytest.mark.parametrize("mode,n", [(0, 5), (1, 4), (0, 2)])
def test_ocv_device_batch_lanes(engine, oracle, synth, pkg, monkeypatch, streams, mode, n):
    """sgm_match_device_batch in the OpenCV modes: frames dealt over same-device stream lanes
    (SGM_OCV_STREAMS; 1 = one after another on the handle's stream) give each frame's own
    result, with median + speckles, and the call stays ordered on the caller's stream."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("SGM_OCV_STREAMS", streams)
    h, w = 60, 300
    p = pkg.default_params(mode, min_disparity=3, num_disparities=48, block_size=5, speckle_window_size=20)
    engine.set_params(p)
    frames = [synth.stereo_pair(h, w, 3, 48, seed=700 + i) for i in range(n)]
    dl = [torch.from_numpy(f[0]).cuda() for f in frames]
    dr = [torch.from_numpy(f[1]).cuda() for f in frames]
    out = torch.full((n, h, w), 777, dtype=torch.int16, device="cuda")
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    for _ in range(2):                    # twice: the lanes' workspaces are reused
        out.fill_(777)
        stream.wait_stream(torch.cuda.current_stream())
        engine.match_device_batch([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], w, h, w,
                                  [out[i].data_ptr() for i in range(n)], w, stream.cuda_stream)
        with torch.cuda.stream(stream):
            got = out.clone()                 # on the caller's stream: after every lane
        stream.synchronize()
        got = got.cpu().numpy()
        op = to_oracle_params(oracle, p)
        for i, (l, r, _) in enumerate(frames):
            assert np.array_equal(got[i], oracle.match(op, l, r)), f"frame {i}"


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("h,w,minD,D,block,compat", [(48, 600, 0, 144, 5, 7), (40, 640, -7, 208, 9, 0),
                                                     (36, 700, 5, 256, 3, 7), (30, 520, 2, 160, 7, 0)])
@pytest.mark.parametrize("nobuf", ["", "1"], ids=["buf32", "rebased"])
def test_ocv_fused_vertical_32_lane_lines(engine, oracle, synth, pkg, monkeypatch, mode, h, w, minD, D, block, compat,
                                          nobuf):
    """128 < D <= 256 beside the fused vertical WTA (forced here with SGM_OCV_VWTA=1; large frames
    take it by default): the path lines are 32 lanes of 8 values (ocv_lanes_per_line), the packed
    4-dword step with the wave priority, writing deficit records; with SGM_OCV_NO_BUF=1 the
    rebased form of volumes past 4 GiB (one descriptor per half-wave line, k_ocv_paths REBK);
    bit-exact vs the oracle in both modes and compat builds."""
    monkeypatch.setenv("SGM_OCV_VWTA", "1")
    if nobuf:
        monkeypatch.setenv("SGM_OCV_NO_BUF", nobuf)
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=h * D)
    p = pkg.default_params(mode, min_disparity=minD, num_disparities=D, block_size=block, ocv_compat=compat)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", [0, 1])
def test_ocv_1080p_d256_full_frame_vs_oracle(engine, oracle, synth, pkg, mode):
    """A whole 1920 x 1080 D=256 frame on the default choices (MODE_HH: the fused vertical WTA with
    32-lane path lines; MODE_SGBM: the row WTA over deficit records of 16-lane lines), bit for bit
    against the oracle."""
    left, right, _ = synth.stereo_pair(1080, 1920, 0, 256, seed=256, with_truth=False)
    p = pkg.default_params(mode, min_disparity=0, num_disparities=256, block_size=5, speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.timeout(900)
def test_ocv_12mp_d256_hh_rebased_full_frame_vs_oracle(engine, oracle, synth, pkg):
    """A 4096 x 3000 D=256 MODE_HH frame: 5.9 GB volumes, so the 32-lane path lines of 8 values run the
    rebased packed kernel (one descriptor per half-wave line) and write deficit records that the
    fused vertical WTA reads; bit for bit against the oracle."""
    left, right, _ = synth.stereo_pair(3000, 4096, 0, 256, seed=4256, with_truth=False)
    p = pkg.default_params(1, min_disparity=0, num_disparities=256, block_size=5, speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
