"""The reference's own shipped SGBM configuration on the GPU (VERDICT r1 "missing" #2).

launch/stereo_matcher.launch:37-48 (stereo_algorithm 1 = OpenCV SGBM): min_disparity 147,
disparity_range 480, correlation_window_size 21, uniqueness_ratio 2, speckle 1000 / 4,
prefilter_cap 7, P1 200, P2 400; capture size 2448 x 2048 (launch/stereo_capture.launch:14-15).
The setters reach cv::StereoSGBM unchanged (matcherOpenCVSGBM.cpp:53-110, via
generate_disparity.cpp:241-261). With a 21 x 21 box at ftzero 15 a cost may leave int16
(bound 441 * 93 + 400 = 41 413), so the engine runs gated: the cost kernel flags the C'
values that do, and only then do the int32 volumes run (Geom::wide == 2).

The processing launch (launch/stereo_processing.launch:65-66, stereo_algorithm 1) keeps those
values and searches minD 0, D 752 instead: D > 512 takes the full int16 path volumes (no 9-bit
deficits), 64-bit offsets (a 5.2 GB volume is past the 32-bit buffer range) and 64-lane path
lines with 16 values per lane whose last active lane straddles D (752 % 32 = 16).
"""
import os

import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu

REF_W, REF_H = 2448, 2048
REF_KW = dict(min_disparity=147, num_disparities=480, block_size=21, uniqueness_ratio=2, speckle_window_size=1000,
              speckle_range=4, prefilter_cap=7, p1=200, p2=400)


def _params(pkg, mode):
    return pkg.default_params(pkg.MODE_OCV_SGBM5 if mode == "sgbm" else pkg.MODE_OCV_HH8, **REF_KW)


PROC_KW = dict(REF_KW, min_disparity=0, num_disparities=752)


@pytest.fixture(scope="module")
def ref_frame(synth):
    return synth.stereo_pair(REF_H, REF_W, 147, 480, seed=2448)


@pytest.fixture(scope="module")
def proc_frame(synth):
    return synth.stereo_pair(REF_H, REF_W, 0, 752, seed=752)


@pytest.mark.parametrize("mode", ["sgbm", "hh"])
def test_reference_config_full_width_crop_vs_oracle(engine, oracle, pkg, ref_frame, mode, monkeypatch):
    """A full-width 2448 x 160 crop of the capture-size frame: bit-exact vs the oracle, in the
    gated mode (no C' leaves int16 on this image: int16 volumes) and with the int32 volumes
    forced (SGM_OCV_GATE=0, the static choice)."""
    left, right, _ = ref_frame
    l, r = np.ascontiguousarray(left[600:760]), np.ascontiguousarray(right[600:760])
    p = _params(pkg, mode)
    engine.set_params(p)
    ref = oracle.match(to_oracle_params(oracle, p), l, r)
    got = engine.match(l, r)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
    monkeypatch.setenv("SGM_OCV_GATE", "0")
    got32 = engine.match(l, r)
    assert np.array_equal(got32, ref), f"int32 volumes: {(got32 != ref).sum()} pixels differ"
    assert (ref != (147 - 1) * 16).mean() > 0.3          # the crop is mostly matched


@pytest.mark.parametrize("mode", ["sgbm", "hh"])
def test_reference_config_gate_takes_int32_on_overflow(engine, oracle, pkg, mode):
    """Same box and P2, a frame whose costs do leave int16 (binary noise against its negative at
    preFilterCap 63): the flag routes it to the int32 volumes, bit-exact vs the oracle (an int16
    path would differ)."""
    rng = np.random.default_rng(1)
    left = (rng.integers(0, 2, (64, 900)) * 255).astype(np.uint8)
    right = 255 - left
    p = pkg.default_params(pkg.MODE_OCV_SGBM5 if mode == "sgbm" else pkg.MODE_OCV_HH8,
                           **dict(REF_KW, prefilter_cap=63, speckle_window_size=0))
    engine.set_params(p)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    got = engine.match(left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["sgbm", "hh"])
def test_reference_config_full_frame_vs_oracle(engine, oracle, pkg, ref_frame, mode):
    """The whole shipped 2448 x 2048 frame (minD 147, D 480, block 21) under the default melodic
    build against the oracle, bit for bit: the default path end to end at its production size —
    the fused cost kernel's full band / strip layout (k_ocv_cost_fused<21, 16, 4>), the 32-bit
    buffer-offset path kernel over 3.6 GB volumes, the fused vertical path + WTA, median and
    speckles. (The oracle takes about a minute per mode here.)"""
    left, right, _ = ref_frame
    p = _params(pkg, mode)
    assert p.ocv_compat == pkg.COMPAT_MELODIC
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
    assert (ref != (147 - 1) * 16).mean() > 0.5


@pytest.mark.parametrize("mode", ["sgbm", "hh"])
def test_reference_config_full_frame_properties(engine, pkg, ref_frame, mode, monkeypatch):
    """The whole 2448 x 2048 frame (the CPU oracle takes minutes at this size): repeatable,
    identical through the gated int16 volumes (3.6 GB each: the 32-bit buffer-offset path
    kernel), the same with 64-bit addresses (SGM_OCV_NO_BUF=1) and the forced int32 volumes,
    inside the search window and close to the synthetic truth."""
    left, right, truth = ref_frame
    p = _params(pkg, mode)
    engine.set_params(p)
    a = engine.match(left, right)
    b = engine.match(left, right)
    assert np.array_equal(a, b)
    monkeypatch.setenv("SGM_OCV_GATE", "0")
    c = engine.match(left, right)
    assert np.array_equal(a, c), f"gated vs int32 volumes: {(a != c).sum()} pixels differ"
    monkeypatch.delenv("SGM_OCV_GATE")
    monkeypatch.setenv("SGM_OCV_NO_BUF", "1")
    d = engine.match(left, right)
    assert np.array_equal(a, d), f"buffer offsets vs 64-bit addresses: {(a != d).sum()} pixels differ"
    valid = a != (147 - 1) * 16
    assert valid.mean() > 0.5
    err = np.abs(a[valid] / 16.0 - truth[valid])
    assert np.median(err) < 0.5 and (err < 2).mean() > 0.9, (np.median(err), (err < 2).mean())
    # disparities inside the search window
    v = a[valid]
    assert v.min() >= 147 * 16 and v.max() <= (147 + 480) * 16


@pytest.mark.parametrize("compat", [0, 7], ids=["scalar-int32", "melodic-int16"])
def test_reference_config_hh_device_batch(engine, pkg, ref_frame, compat):
    """The shipped 2448 x 2048 D=480 block-21 frame in MODE_HH through sgm_match_device_batch
    with 5 frames: the same-device stream lanes are opened only while the free HBM
    holds their workspaces (scalar build: int32 volumes, ~70 GB each; melodic: int16), with the
    handle itself as lane 0; every frame equals its single match."""
    torch = pytest.importorskip("torch")
    left, right, _ = ref_frame
    p = pkg.default_params(pkg.MODE_OCV_HH8, ocv_compat=compat, **REF_KW)
    engine.set_params(p)
    n = 5
    ls = [np.ascontiguousarray(np.roll(left, 7 * i, axis=0)) for i in range(n)]
    rs = [np.ascontiguousarray(np.roll(right, 7 * i, axis=0)) for i in range(n)]
    dl = [torch.from_numpy(a).cuda() for a in ls]
    dr = [torch.from_numpy(a).cuda() for a in rs]
    out = torch.full((n, REF_H, REF_W), 777, dtype=torch.int16, device="cuda")
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    engine.match_device_batch([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], REF_W, REF_H, REF_W,
                              [out[i].data_ptr() for i in range(n)], REF_W, stream.cuda_stream)
    stream.synchronize()
    got = out.cpu().numpy()
    del out, dl, dr
    for i in (0, n - 1):
        single = engine.match(ls[i], rs[i])
        assert np.array_equal(got[i], single), f"frame {i}: {(got[i] != single).sum()} pixels differ"


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["sgbm", "hh"])
def test_processing_config_full_frame_vs_oracle(engine, oracle, pkg, proc_frame, mode, monkeypatch):
    """The processing launch's matcher (stereo_processing.launch:65-66: minD 0, D 752; block 21,
    uniqueness 2, speckle 1000 / 4, cap 7, P1 200, P2 400 from stereo_matcher.launch:39-47) on a
    whole 2448 x 2048 frame under the default melodic build, bit for bit against the oracle
    (VERDICT r5 #1): five or eight full int16 volumes of 5.2 GB each, 64-bit path offsets, the
    straddling lane, median and speckles; then the same frame with the int32 volumes forced
    (SGM_OCV_GATE=0, 10.4 GB each) equals it. (The oracle takes 1-2 minutes per mode.)"""
    left, right, truth = proc_frame
    p = pkg.default_params(pkg.MODE_OCV_SGBM5 if mode == "sgbm" else pkg.MODE_OCV_HH8, **PROC_KW)
    assert p.ocv_compat == pkg.COMPAT_MELODIC
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
    valid = ref != -16
    assert valid.mean() > 0.5
    err = np.abs(ref[valid] / 16.0 - truth[valid])
    assert np.median(err) < 0.5, np.median(err)
    monkeypatch.setenv("SGM_OCV_GATE", "0")
    got32 = engine.match(left, right)
    assert np.array_equal(got32, ref), f"int32 volumes: {(got32 != ref).sum()} pixels differ"


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["sgbm", "hh"])
def test_capture_size_d512_full_frame_vs_oracle(engine, oracle, pkg, synth, mode):
    """The capture size with D = 512 from minD 0 (the launch values with a range just past the shipped
    480): 4.06 GB int16 volumes, the largest a 64-lane line of 8 values meets at this size and just
    below the 32-bit buffer range (4.29 GB: the buffer offsets run to within 6 % of their wrap),
    deficit records through the fused vertical WTA; bit for bit against the oracle."""
    left, right, _ = synth.stereo_pair(REF_H, REF_W, 0, 512, seed=512)
    p = pkg.default_params(pkg.MODE_OCV_SGBM5 if mode == "sgbm" else pkg.MODE_OCV_HH8, **dict(PROC_KW, num_disparities=512))
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
    assert (ref != -16).mean() > 0.5


@pytest.mark.timeout(1100)
def test_12mp_d480_rebased_full_frame_vs_oracle(engine, oracle, pkg, synth):
    """A 4096 x 3000 D=480 MODE_SGBM frame: 10.4 GB int16 volumes, so 64-lane lines of 8 values run
    the step-rebased packed kernel (REBK) with deficit records and the fused vertical WTA reads them;
    bit for bit against the oracle (the single-threaded restatement takes about a minute on the box)."""
    left, right, _ = synth.stereo_pair(3000, 4096, 0, 480, seed=4096, with_truth=False)
    p = pkg.default_params(pkg.MODE_OCV_SGBM5, min_disparity=0, num_disparities=480, block_size=5,
                           speckle_window_size=0)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
