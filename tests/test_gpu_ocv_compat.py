"""GPU parity of the OpenCV build variants (`sgm_params.ocv_compat`, include/sgm_hip.h SGM_OCV_*).

The reference pins OpenCV only by ROS distro: its Dockerfile (Dockerfile:1, amd64) is melodic,
i.e. OpenCV 3.2 with the SSE2 branches of computeDisparitySGBM, and its CI also builds noetic
(OpenCV 4.2, universal intrinsics; .github/workflows/ros-build.yml:14-21). The oracle restates
the three known divergences as switches (oracle/sgm_oracle.c): COL0_LEGACY (1),
SIMD_SAT (2), LANE_TIE (4). Here the engine runs every combination bit-exactly against the
oracle on BASELINE configs[0] (C1), on 1920x1080, on the reference's shipped configuration
(launch/stereo_matcher.launch:37-48) and on frames in the overflow regime, where the SIMD builds
take the sequential saturating cost and saturating int16 paths (ocv_sgm.hip, Geom::wide).
"""
import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu

ALL = list(range(8))
REF_KW = dict(min_disparity=147, num_disparities=480, block_size=21, uniqueness_ratio=2, speckle_window_size=1000,
              speckle_range=4, prefilter_cap=7, p1=200, p2=400)


def _check(engine, oracle, p, left, right):
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"compat {p.ocv_compat}: {(got != ref).sum()} pixels differ"
    return ref


@pytest.fixture(scope="module")
def c1_pair(synth):
    return synth.stereo_pair(480, 640, 9, 64, seed=640)


@pytest.mark.parametrize("compat", ALL)
@pytest.mark.parametrize("mode", [0, 1])
def test_compat_c1_node_defaults(engine, oracle, pkg, c1_pair, mode, compat):
    """BASELINE configs[0]: 640x480, the node defaults (generate_disparity.cpp:100-112) +
    median + speckle, every variant."""
    left, right, _ = c1_pair
    _check(engine, oracle, pkg.default_params(mode, ocv_compat=compat), left, right)


def test_compat_default_is_melodic(engine, oracle, pkg, c1_pair):
    """sgm_default_params picks the melodic build (the reference's Docker image); its column-0
    rule makes it differ from the scalar restatement on every frame."""
    left, right, _ = c1_pair
    p = pkg.default_params(pkg.MODE_OCV_SGBM5)
    assert p.ocv_compat == pkg.COMPAT_MELODIC == 7
    mel = _check(engine, oracle, p, left, right)
    sca = _check(engine, oracle, p.copy(ocv_compat=0), left, right)
    assert not np.array_equal(mel, sca)


@pytest.fixture(scope="module")
def hd_pair(synth):
    return synth.stereo_pair(1080, 1920, 0, 128, seed=1080)


@pytest.mark.parametrize("compat", ALL)
@pytest.mark.parametrize("mode", [0, 1])
def test_compat_1080p(engine, oracle, pkg, hd_pair, mode, compat):
    """1920x1080 D=128 block 5, MODE_SGBM and MODE_HH (oracle: single-threaded, seconds)."""
    left, right, _ = hd_pair
    p = pkg.default_params(mode, min_disparity=0, num_disparities=128, block_size=5, speckle_window_size=0,
                           ocv_compat=compat)
    _check(engine, oracle, p, left, right)


@pytest.fixture(scope="module")
def ref_crop(synth):
    left, right, _ = synth.stereo_pair(2048, 2448, 147, 480, seed=2448)
    return np.ascontiguousarray(left[600:760]), np.ascontiguousarray(right[600:760])


@pytest.mark.parametrize("compat", [0, 1, 2, 4, 7])
@pytest.mark.parametrize("mode", [0, 1])
def test_compat_shipped_config_crop(engine, oracle, pkg, ref_crop, mode, compat):
    """The reference's launch configuration (min 147, D 480, block 21, cap 7, P1 200 / P2 400)
    on a full-width 2448 x 160 crop of the capture-size frame: in the gated overflow regime
    (box bound 441 * 77 + 400 > 32767 - 400), no C' actually leaves the plain kernels' range."""
    left, right = ref_crop
    p = pkg.default_params(mode, ocv_compat=compat, **REF_KW)
    ref = _check(engine, oracle, p, left, right)
    assert (ref != (147 - 1) * 16).mean() > 0.3


def _binary(h, w, seed):
    rng = np.random.default_rng(seed)
    left = (rng.integers(0, 2, (h, w)) * 255).astype(np.uint8)
    return left, 255 - left


@pytest.mark.parametrize("compat", ALL)
@pytest.mark.parametrize("mode", [0, 1])
def test_compat_overflow_frame(engine, oracle, pkg, mode, compat):
    """The shipped box and P2 at preFilterCap 63 on binary noise against its negative: box sums
    pass 32767, so the scalar builds take the int32 volumes and the SIMD ones the saturating
    kernels (the two results differ, test_oracle_ocv_variants.py)."""
    left, right = _binary(64, 900, 1)
    p = pkg.default_params(mode, ocv_compat=compat, **dict(REF_KW, prefilter_cap=63, speckle_window_size=0))
    _check(engine, oracle, p, left, right)


@pytest.mark.parametrize("chain", ["sat2", "seq"])
@pytest.mark.parametrize("compat", [0, 1, 2, 3])
@pytest.mark.parametrize("mode", [0, 1])
def test_compat_cost_volume_overflow(engine, oracle, pkg, monkeypatch, mode, compat, chain):
    """C' itself on the overflow frame (sgm_debug_ocv_cost): the wrapped scalar volume, or the
    SIMD builds' saturated running sums — from the vertical saturating update over the plain
    horizontal sums (k_ocv_vsum_sat2, the default) and from the sequential chain it replaced
    (SGM_OCV_SAT_SEQ=1)."""
    if chain == "seq":
        monkeypatch.setenv("SGM_OCV_SAT_SEQ", "1")
    left, right = _binary(64, 160, 1)
    p = pkg.default_params(mode, min_disparity=0, num_disparities=64, block_size=21, prefilter_cap=63, p1=50,
                           p2=3000, speckle_window_size=0, ocv_compat=compat)
    engine.set_params(p)
    got = engine.ocv_cost(left, right)
    ref = oracle.ocv_cost(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} cells differ"
    if compat & 2:
        assert (ref == 32767).any()


@pytest.mark.parametrize("mode", [0, 1])
def test_compat_cost_volume_saturating_hsum(engine, oracle, pkg, mode):
    """A box wide enough for the SIMD horizontal running sums to saturate too (181 columns x
    (2*63 + 63) > 32767): the sequential chain keeps the SIMD branch exact there."""
    rng = np.random.default_rng(7)
    left = (rng.integers(0, 2, (200, 260)) * 255).astype(np.uint8)
    right = 255 - left
    for compat in (2, 7):
        p = pkg.default_params(mode, min_disparity=0, num_disparities=16, block_size=181, prefilter_cap=63, p1=50,
                               p2=3000, speckle_window_size=0, ocv_compat=compat)
        engine.set_params(p)
        got = engine.ocv_cost(left, right)
        ref = oracle.ocv_cost(to_oracle_params(oracle, p), left, right)
        assert np.array_equal(got, ref), f"compat {compat}: {(got != ref).sum()} cells differ"
        assert (ref == 32767).any()


@pytest.fixture(scope="module")
def full_overflow_pair():
    """A capture-size (2448 x 2048) high-contrast frame: binary noise against its negative."""
    return _binary(2048, 2448, 11)


OVF_KW = dict(REF_KW, prefilter_cap=63, p2=4000, speckle_window_size=0)   # cfg maxima: C' passes 32767


@pytest.mark.timeout(900)
def test_compat_full_size_overflow_cost_volume(engine, oracle, pkg, full_overflow_pair):
    """C' of a full 2448 x 2048 frame at the shipped geometry (min 147, D 480, block 21) in the
    overflow regime (cap 63, P2 4000: box sums + P2 pass 32767), melodic and noetic (the SIMD
    builds: saturating vertical sums) and the scalar build (wrapping), against the oracle."""
    left, right = full_overflow_pair
    sums = {}
    for compat in (7, 2, 0):
        p = pkg.default_params(0, ocv_compat=compat, **OVF_KW)
        engine.set_params(p)
        got = engine.ocv_cost(left, right)
        ref = oracle.ocv_cost(to_oracle_params(oracle, p), left, right)
        assert np.array_equal(got, ref), f"compat {compat}: {(got != ref).sum()} cells differ"
        sums[compat] = int(ref[1:].astype(np.int64).sum())
        if compat == 0:
            assert (ref < 0).any()            # the scalar CostType wraps
        del got, ref
    assert sums[2] != sums[0]                  # the SIMD builds saturate instead


@pytest.mark.timeout(900)
def test_compat_full_size_overflow_frame(engine, oracle, pkg, full_overflow_pair):
    """The same full-size overflow frame matched end to end under the default (melodic) build."""
    left, right = full_overflow_pair
    _check(engine, oracle, pkg.default_params(0, ocv_compat=7, **OVF_KW), left, right)


@pytest.mark.parametrize("mode", [0, 1])
def test_compat_simd_threshold_band(engine, oracle, pkg, mode):
    """A frame whose largest C' is exactly 32767: inside int16 (the scalar build stays on the
    plain int16 kernels) but above 32767 - P2, where the SIMD delta (short)(minLr + P2) can wrap
    — the SIMD build must take its flagged kernels. Both bit-exact."""
    left, right = _binary(48, 400, 3)
    kw = dict(min_disparity=0, num_disparities=48, block_size=15, prefilter_cap=40, p1=30, speckle_window_size=0,
              uniqueness_ratio=0)
    probe = oracle.make_params(mode, p2=100, ocv_compat=0, **kw)
    box_max = int(oracle.ocv_cost(probe, left, right).max()) - 100
    p2 = 32767 - box_max
    assert 2 * p2 > 32767 - box_max > 0
    for compat in (0, 2):
        _check(engine, oracle, pkg.default_params(mode, p2=p2, ocv_compat=compat, **kw), left, right)


def test_compat_lane_tie_periodic_texture(engine, oracle, pkg):
    """A 9-periodic texture ties S(d) and S(d + 9) across SSE2 lanes: the 3.x lane rule moves
    MODE_SGBM winners (not MODE_HH's) — bit-exact on the GPU either way."""
    rng = np.random.default_rng(4)
    tile = rng.integers(0, 256, (64, 9), dtype=np.uint8)
    left = np.tile(tile, (1, 24))[:, :200].copy()
    right = np.roll(left, -7, axis=1)
    res = {}
    for mode in (0, 1):
        for compat in (0, 4):
            p = pkg.default_params(mode, min_disparity=0, num_disparities=32, uniqueness_ratio=0, block_size=3,
                                   speckle_window_size=0, ocv_compat=compat)
            res[mode, compat] = _check(engine, oracle, p, left, right)
    assert not np.array_equal(res[0, 0], res[0, 4])
    assert np.array_equal(res[1, 0], res[1, 4])


@pytest.mark.parametrize("compat", [0, 7])
def test_compat_device_batch_lanes(engine, oracle, synth, pkg, compat):
    """sgm_match_device_batch (same-device stream lanes) keeps each frame's variant result."""
    torch = pytest.importorskip("torch")
    h, w, n = 60, 300, 4
    p = pkg.default_params(0, min_disparity=3, num_disparities=48, block_size=5, speckle_window_size=20,
                           ocv_compat=compat)
    engine.set_params(p)
    frames = [synth.stereo_pair(h, w, 3, 48, seed=900 + i) for i in range(n - 1)] + [_binary(h, w, 5) + (None,)]
    dl = [torch.from_numpy(f[0]).cuda() for f in frames]
    dr = [torch.from_numpy(f[1]).cuda() for f in frames]
    out = torch.full((n, h, w), 777, dtype=torch.int16, device="cuda")
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    engine.match_device_batch([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], w, h, w,
                              [out[i].data_ptr() for i in range(n)], w, stream.cuda_stream)
    stream.synchronize()
    got = out.cpu().numpy()
    op = to_oracle_params(oracle, p)
    for i, f in enumerate(frames):
        assert np.array_equal(got[i], oracle.match(op, f[0], f[1])), f"frame {i}"
