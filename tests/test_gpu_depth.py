"""GPU parity: DisparityImage packing and disparity -> depth / point cloud, bit-exact
against the oracle's float32 restatements (disparity_to_depth.cpp:127-205,
generate_disparity.cpp:426-452)."""
import numpy as np
import pytest

from test_depth_oracle import _q, _sample_disp

pytestmark = pytest.mark.gpu


def _stream(torch):
    """A side stream ordered after torch's queued work (the library's NULL stream argument
    means the handle's own stream)."""
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    _stream.keep.append(st)
    return st.cuda_stream


_stream.keep = []


def _dev(torch, a):
    return torch.as_tensor(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("shape", [(1, 1), (7, 300), (61, 129)])
def test_disparity_to_msg(engine, oracle, shape):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(shape[0] * 31 + shape[1])
    h, w = shape
    d16 = rng.integers(-300, 4000, (h, w)).astype(np.int16)
    src = _dev(torch, d16)
    out = torch.full((h, w + 5), -1.0, dtype=torch.float32, device="cuda")
    for lo, hi in [(0.0, float("inf")), (2.0, 150.0)]:
        engine.disparity_to_msg(src.data_ptr(), w, w, h, lo, hi, out.data_ptr(), w + 5,
                                _stream(torch))
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert np.array_equal(got[:, :w].view(np.uint32), oracle.disparity_to_msg(d16, lo, hi).view(np.uint32))
        assert (got[:, w:] == -1).all()


@pytest.mark.parametrize("channels", [0, 1, 3])
@pytest.mark.parametrize("window", [(0.0, 100.0), (0.6, 4.0)])
def test_depth_points(engine, oracle, pkg, channels, window):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(channels * 7 + int(window[1]))
    h, w = 70, 333
    d = _sample_disp(rng, h, w)
    color = None if channels == 0 else rng.integers(0, 256, (h, w) if channels == 1 else (h, w, 3), dtype=np.uint8)
    Q = oracle.calc_q(*_q())
    depth, pts, rgba = pkg.disp_info_to_depth(engine, d, color, Q, *window)
    rd, rp, rr = oracle.depth_points(d, Q, *window, color)
    assert np.array_equal(depth.view(np.uint32), rd.view(np.uint32))
    assert np.array_equal(pts.view(np.uint32), rp.view(np.uint32)), f"{len(pts)} vs {len(rp)} points"
    assert np.array_equal(rgba, rr)


def test_depth_points_truncation_and_count(engine, oracle, pkg):
    """max_points below the number of points: only the first ones (raster order) are written,
    the count is the full total; depth without points."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(11)
    h, w = 40, 90
    d = _sample_disp(rng, h, w)
    Q = oracle.calc_q(*_q())
    rd, rp, _ = oracle.depth_points(d, Q, 0.0, 100.0)
    dd = _dev(torch, d)
    cap = len(rp) // 3
    pts = torch.full((cap + 8, 4), -7.0, dtype=torch.float32, device="cuda")
    n = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = _stream(torch)
    engine.depth_points(dd.data_ptr(), w, w, h, pkg.q_terms(Q), 0.0, 100.0, d_points=pts.data_ptr(), max_points=cap,
                        d_num_points=n.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert int(n.item()) == len(rp)
    got = pts.cpu().numpy()
    assert np.array_equal(got[:cap, :3].view(np.uint32), rp[:cap].view(np.uint32))
    assert (got[cap:] == -7).all()
    depth = torch.zeros((h, w), dtype=torch.float32, device="cuda")
    engine.depth_points(dd.data_ptr(), w, w, h, pkg.q_terms(Q), 0.0, 100.0, d_depth=depth.data_ptr(), depth_stride=w,
                        stream=s)
    torch.cuda.synchronize()
    assert np.array_equal(depth.cpu().numpy().view(np.uint32), rd.view(np.uint32))


def test_match_to_cloud_chain(engine, oracle, pkg, synth):
    """The node chain on the GPU: census match -> DisparityImage -> depth + cloud, at C1 size."""
    torch = pytest.importorskip("torch")
    from conftest import to_oracle_params
    h, w = 480, 640
    left, right, _ = synth.stereo_pair(h, w, 0, 64, seed=21)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=64)
    engine.set_params(p)
    disp16 = engine.match(left, right)
    assert np.array_equal(disp16, oracle.match(to_oracle_params(oracle, p), left, right))
    f, T, zmin, zmax = 712.5, 0.119, 0.5, 20.0
    lo, hi = np.float32(T * f / zmax), np.float32(T * f / zmin)
    src = _dev(torch, disp16)
    msg = torch.empty((h, w), dtype=torch.float32, device="cuda")
    engine.disparity_to_msg(src.data_ptr(), w, w, h, lo, hi, msg.data_ptr(), w, _stream(torch))
    torch.cuda.synchronize()
    m = msg.cpu().numpy()
    assert np.array_equal(m.view(np.uint32), oracle.disparity_to_msg(disp16, lo, hi).view(np.uint32))
    Q = oracle.calc_q(*_q())
    depth, pts, rgba = pkg.disp_info_to_depth(engine, m, left, Q, zmin, zmax)
    rd, rp, rr = oracle.depth_points(m, Q, zmin, zmax, left)
    assert np.array_equal(depth.view(np.uint32), rd.view(np.uint32)) and np.array_equal(rr, rgba)
    assert np.array_equal(pts.view(np.uint32), rp.view(np.uint32)) and len(rp) > 0.3 * h * w
