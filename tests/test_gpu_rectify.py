"""GPU parity: rectification maps (initUndistortRectifyMap CV_32FC1) and the INTER_CUBIC
remap, bit-exact against the oracle's restatements (generate_disparity.cpp:370-386,
rectify.cpp:111-127)."""
import numpy as np
import pytest

from test_rectify_oracle import calib

pytestmark = pytest.mark.gpu


def _maps(torch, engine, K, D, R, P, w, h, stride=None):
    stride = stride or w
    mx = torch.full((h, stride), -7.0, dtype=torch.float32, device="cuda")
    my = torch.full((h, stride), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()       # NULL stream argument = the handle's stream, not torch's
    engine.rectify_map(K, D, R, P, w, h, mx.data_ptr(), my.data_ptr(), stride)
    engine.synchronize()
    return mx, my


@pytest.mark.parametrize("w,h,nd,stride", [(640, 480, 5, 640), (333, 217, 0, 340), (96, 64, 4, 96),
                                           (128, 80, 8, 128), (200, 100, 12, 203), (1920, 1080, 5, 1920)])
def test_rectify_map_bit_exact(engine, oracle, w, h, nd, stride):
    torch = pytest.importorskip("torch")
    K, D, R, P = calib(seed=w + nd, w=w, h=h)
    Dn = np.concatenate([D, [0.01, -0.002, 0.0005, 0.001, -0.0007, 0.0003, 0.0002]])[:nd]
    mx, my = _maps(torch, engine, K, Dn, R, P, w, h, stride)
    rx, ry = oracle.rectify_map(K, Dn, R, P, w, h)
    gx, gy = mx.cpu().numpy(), my.cpu().numpy()
    assert np.array_equal(gx[:, :w].view(np.uint32), rx.view(np.uint32))
    assert np.array_equal(gy[:, :w].view(np.uint32), ry.view(np.uint32))
    assert (gx[:, w:] == -7).all() and (gy[:, w:] == -7).all()


def test_rectify_map_identity_rotation_none(engine, oracle):
    torch = pytest.importorskip("torch")
    K, D, _, P = calib(seed=1, w=160, h=120, rot=False)
    mx, my = _maps(torch, engine, K, D, None, P, 160, 120)
    rx, ry = oracle.rectify_map(K, D, None, P, 160, 120)
    assert np.array_equal(mx.cpu().numpy().view(np.uint32), rx.view(np.uint32))
    assert np.array_equal(my.cpu().numpy().view(np.uint32), ry.view(np.uint32))


def test_rectify_map_errors(engine, pkg):
    torch = pytest.importorskip("torch")
    K, D, R, P = calib(w=32, h=16)
    m = torch.empty((16, 32), dtype=torch.float32, device="cuda")
    with pytest.raises(pkg.SGMError):
        engine.rectify_map(K, np.zeros(14), R, P, 32, 16, m.data_ptr(), m.data_ptr(), 32)
    with pytest.raises(pkg.SGMError):
        engine.rectify_map(K, D, R, np.zeros((3, 4)), 32, 16, m.data_ptr(), m.data_ptr(), 32)
    with pytest.raises(pkg.SGMError):
        engine.rectify_map(K, D, R, P, 32, 16, m.data_ptr(), m.data_ptr(), 31)


@pytest.mark.parametrize("sw,sh,w,h", [(31, 23, 27, 19), (640, 480, 640, 480), (300, 200, 350, 170), (3, 2, 9, 7)])
def test_remap_cubic_random_maps(engine, oracle, sw, sh, w, h):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(sw * 7 + h)
    src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
    mx = rng.uniform(-6, sw + 6, (h, w)).astype(np.float32)
    my = rng.uniform(-6, sh + 6, (h, w)).astype(np.float32)
    mx[0, :4] = [np.nan, np.inf, -1e12, 3.015625]
    my[min(1, h - 1), :2] = [1e30, 0.515625]
    mx[h // 2] = np.round(mx[h // 2] * 64) / 64            # exact 1/64 ties (round half to even)
    d_src = torch.as_tensor(src).cuda()
    d_mx, d_my = torch.as_tensor(mx).cuda(), torch.as_tensor(my).cuda()
    out = torch.full((h, w + 3), 99, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    engine.remap_cubic(d_src.data_ptr(), sw, sw, sh, d_mx.data_ptr(), d_my.data_ptr(), w, w, h, out.data_ptr(),
                       w + 3)
    engine.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(got[:, :w], oracle.remap_cubic(src, mx, my))
    assert (got[:, w:] == 99).all()


@pytest.mark.parametrize("w,h", [(640, 480), (1920, 1080)])
def test_rectify_end_to_end(engine, oracle, pkg, synth, w, h):
    """The node's rectify(): map + remap of a textured frame equals the oracle chain, and the
    cached maps give the same result on the next frame."""
    K, D, R, P = calib(seed=9, w=w, h=h)
    left, right, _ = synth.stereo_pair(h, w, 0, 64, seed=w)
    got, maps = pkg.rectify(engine, left, K, D, R, P)
    rx, ry = oracle.rectify_map(K, D, R, P, w, h)
    assert np.array_equal(got, oracle.remap_cubic(left, rx, ry))
    got2, _ = pkg.rectify(engine, right, K, D, R, P, maps=maps)
    assert np.array_equal(got2, oracle.remap_cubic(right, rx, ry))


def _raw_pair(synth, h, w, seed):
    left, right, _ = synth.stereo_pair(h, w, 0, 48, seed=seed)
    return left, right


@pytest.mark.parametrize("n,raw,rect", [(1, (480, 640), (480, 640)), (3, (500, 700), (432, 608)),
                                        (5, (240, 320), (240, 320))])
def test_fused_rectify_census_batch(engine, oracle, pkg, synth, n, raw, rect):
    """sgm_set_rectification + sgm_match_device_batch_rect: raw frames are rectified inside the
    census tiles; the disparities equal the oracle's match of the oracle-rectified pair and
    the rectified images equal the oracle remap (bit-exact)."""
    torch = pytest.importorskip("torch")
    from conftest import to_oracle_params
    (rh, rw), (h, w) = raw, rect
    KL, DL, RL, PL = calib(seed=11, w=rw, h=rh)
    KR, DR, RR, PR = calib(seed=12, w=rw, h=rh)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=64)
    engine.set_params(p)
    mxl, myl = _maps(torch, engine, KL, DL, RL, PL, w, h)
    mxr, myr = _maps(torch, engine, KR, DR, RR, PR, w, h)
    frames = [_raw_pair(synth, rh, rw, 70 + i) for i in range(n)]
    dl = [torch.as_tensor(f[0]).cuda() for f in frames]
    dr = [torch.as_tensor(f[1]).cuda() for f in frames]
    out = torch.full((n, h, w), 777, dtype=torch.int16, device="cuda")
    recl = torch.zeros((n, h, w + 8), dtype=torch.uint8, device="cuda")
    recr = torch.zeros((n, h, w + 8), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    engine.set_rectification((mxl.data_ptr(), myl.data_ptr()), (mxr.data_ptr(), myr.data_ptr()), w, rw, rh)
    try:
        engine.match_device_batch_rect([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], w, h, rw,
                                       [recl[i].data_ptr() for i in range(n)], [recr[i].data_ptr() for i in range(n)],
                                       w + 8, [out[i].data_ptr() for i in range(n)], w)
        engine.synchronize()
        if n == 1:   # the single-frame device entry point takes raw frames too while rectification is on
            one = torch.full((h, w), 555, dtype=torch.int16, device="cuda")
            torch.cuda.synchronize()
            engine.match_device(dl[0].data_ptr(), dr[0].data_ptr(), w, h, rw, one.data_ptr(), w)
            engine.synchronize()
        with pytest.raises(pkg.SGMError):          # host-buffer matches are not rectified
            engine.match(np.zeros((h, w), np.uint8), np.zeros((h, w), np.uint8))
    finally:
        engine.set_rectification()
    rxl, ryl = oracle.rectify_map(KL, DL, RL, PL, w, h)
    rxr, ryr = oracle.rectify_map(KR, DR, RR, PR, w, h)
    op = to_oracle_params(oracle, p)
    got, gl, gr = out.cpu().numpy(), recl.cpu().numpy(), recr.cpu().numpy()
    for i, (l_raw, r_raw) in enumerate(frames):
        el, er = oracle.remap_cubic(l_raw, rxl, ryl), oracle.remap_cubic(r_raw, rxr, ryr)
        assert np.array_equal(gl[i, :, :w], el) and np.array_equal(gr[i, :, :w], er), f"frame {i} rectified"
        assert (gl[i, :, w:] == 0).all()
        assert np.array_equal(got[i], oracle.match(op, el, er)), f"frame {i} disparity"
    if n == 1:
        assert np.array_equal(one.cpu().numpy(), got[0])
