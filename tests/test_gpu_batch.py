"""Host-buffer frame batch (sgm_match_batch, SURVEY §8(e) "frame batch", BASELINE C4).

The batch streams each device's frames through pinned rings (packer thread -> H2D ->
pipelined census batch -> D2H -> unpacker thread). Every frame must equal the single-frame
sgm_match bit for bit, and sampled frames the CPU oracle. Reference pattern: the per-frame
upload / match / download of matcherOpenCVBlockCuda.cpp:27-30, driven by
generate_disparity.cpp:334-368.
"""
import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu


def _c3_params(pkg):
    return pkg.default_params(pkg.MODE_CENSUS8, num_disparities=256, min_disparity=0, p1=10, p2=120,
                              uniqueness_ratio=5, subpixel=1, lr_check=1, disp12_max_diff=1, median=0,
                              speckle_window_size=0)


@pytest.fixture(scope="module")
def c3_frames(synth):
    """8 distinct full 1920x1080 pairs (D = 256 truth range)."""
    return [synth.stereo_pair(1080, 1920, 0, 256, seed=500 + i, with_truth=False)[:2] for i in range(8)]


@pytest.mark.parametrize("devices,n", [([0] * 8, 16), ([0], 20)])
def test_host_batch_c3_full_frames(engine, pkg, oracle, c3_frames, devices, n):
    """>= 16 full C3 frames (BASELINE C4 shape) through sgm_match_batch: 8 device handles
    (2 frames each, one pipelined group) and 1 handle (20 frames: 10 groups, the 8-frame
    rings wrap twice). Each frame == single-frame sgm_match; two frames == the oracle."""
    p = _c3_params(pkg)
    engine.set_params(p)
    lefts = [c3_frames[i % 8][0] for i in range(n)]
    rights = [c3_frames[(i * 3) % 8][1] for i in range(n)]     # mixed pairs: every frame differs
    outs = engine.match_batch(lefts, rights, devices=devices)
    single = {}
    for i in range(n):
        key = (i % 8, (i * 3) % 8)
        if key not in single:
            single[key] = engine.match(lefts[i], rights[i])
        assert np.array_equal(outs[i], single[key]), f"frame {i} differs from sgm_match"
    op = to_oracle_params(oracle, p)
    for i in (0, n - 1):
        assert np.array_equal(outs[i], oracle.match(op, lefts[i], rights[i])), f"frame {i} differs from the oracle"


@pytest.mark.parametrize("mode", ["census", "sgbm5", "hh8"])
def test_host_batch_strided_ring_wrap(engine, pkg, oracle, synth, mode):
    """Row-strided inputs and outputs (stride > width), 21 frames on one handle (rings wrap,
    odd tail group), every mode; results written in place into the strided outputs."""
    h, w, D = 72, 200, 48 if mode == "census" else 32
    if mode == "census":
        p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, min_disparity=0, median=1)
    else:
        p = pkg.default_params(pkg.MODE_OCV_SGBM5 if mode == "sgbm5" else pkg.MODE_OCV_HH8,
                               num_disparities=D, min_disparity=2, block_size=5)
    engine.set_params(p)
    n = 21
    pairs = [synth.stereo_pair(h, w, 0, D, seed=900 + i)[:2] for i in range(n)]
    bigL = np.zeros((n, h, w + 37), np.uint8)
    bigR = np.zeros((n, h, w + 37), np.uint8)
    for i, (l, r) in enumerate(pairs):
        bigL[i, :, :w], bigR[i, :, :w] = l, r
    outbuf = np.full((n, h, w + 11), 7777, np.int16)
    outs = [outbuf[i, :, :w] for i in range(n)]
    engine.match_batch([bigL[i, :, :w] for i in range(n)], [bigR[i, :, :w] for i in range(n)], devices=[0],
                       outs=outs)
    assert (outbuf[:, :, w:] == 7777).all(), "wrote past the output row"
    op = to_oracle_params(oracle, p)
    for i in (0, 9, n - 1):
        assert np.array_equal(outbuf[i, :, :w], oracle.match(op, *pairs[i])), f"frame {i}"
    for i in range(n):
        assert np.array_equal(outbuf[i, :, :w], engine.match(*pairs[i])), f"frame {i} vs sgm_match"


def test_async_calls_on_two_streams(engine, pkg, synth):
    """device calls on different caller streams (and a synchronous call after
    them) share the handle's workspace; each call is ordered after the previous one."""
    torch = pytest.importorskip("torch")
    h, w, D = 256, 640, 128
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D)
    engine.set_params(p)
    pairs = [synth.stereo_pair(h, w, 0, D, seed=70 + i)[:2] for i in range(3)]
    refs = [engine.match(l, r) for l, r in pairs]
    dev = [(torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()) for l, r in pairs]
    outs = [torch.empty((h, w), dtype=torch.int16, device="cuda") for _ in pairs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for rep in range(4):
        for i in range(2):
            engine.match_device(dev[i][0].data_ptr(), dev[i][1].data_ptr(), w, h, w, outs[i].data_ptr(), w,
                                streams[i].cuda_stream)
        # a synchronous host call right behind the two asynchronous ones
        assert np.array_equal(engine.match(*pairs[2]), refs[2])
        torch.cuda.synchronize()
        for i in range(2):
            assert np.array_equal(outs[i].cpu().numpy(), refs[i]), f"rep {rep} stream {i}"


@pytest.mark.parametrize("mode", [0, 2])
def test_match_f32_host_rows(engine, pkg, synth, mode):
    """sgm_match_f32 (the adapter's CV_32FC1 path, converted on the device) equals sgm_match's
    int16 as float, with row-strided host inputs and output (2-D DMAs, no staging)."""
    h, w = 90, 300
    left, right, _ = synth.stereo_pair(h, w, 0, 64, seed=31)
    p = pkg.default_params(mode, min_disparity=0, num_disparities=64, block_size=5)
    engine.set_params(p)
    ref = engine.match(left, right)
    big_l = np.zeros((h, w + 37), np.uint8)
    big_r = np.zeros((h, w + 37), np.uint8)
    big_l[:, 5:5 + w] = left
    big_r[:, 5:5 + w] = right
    out = np.full((h, w + 11), -1.0, np.float32)
    lib = pkg.load_library()
    rc = lib.sgm_match_f32(engine.h, pkg._ptr(big_l[:, 5:]), pkg._ptr(big_r[:, 5:]), w, h, w + 37,
                           pkg._ptr(out), w + 11)
    assert rc == 0, engine.error()
    assert np.array_equal(out[:, :w], ref.astype(np.float32))
    assert (out[:, w:] == -1.0).all()                     # nothing written past the row
    assert np.array_equal(engine.match_f32(left, right), ref.astype(np.float32))
