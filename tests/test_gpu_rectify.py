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
