"""GPU parity — seeded random configurations against the oracle, bit-exact.

Each case draws a mode (census, MODE_SGBM, MODE_HH), an image size (including heights below
the SAD window and widths that leave no valid column), a disparity window (negative minD
included), penalties, uniqueness (0, ordinary, >= 100), LR / subpixel / median / speckle
settings and an image kind (textured stereo pair, noise, or pairs with flat patches that
trip the uniqueness and speckle rules); OpenCV-mode cases also draw the OpenCV build variant
(`ocv_compat`, all eight bit combinations) and sometimes binary 0/255 images whose box sums
leave int16 (the overflow regime: int32 or saturating SIMD kernels). The seeds are fixed, so a failure names a
reproducible configuration. Census cases also run through the pipelined device batch
(`sgm_match_device_batch`) with a random frame count and through the exact row-band mode
(`sgm_match_tiled_exact`) with a random band count.
"""
import os

import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu

N_CASES = int(os.environ.get("SGM_FUZZ_CASES", "120"))   # a longer hunt: SGM_FUZZ_CASES=1000


def _images(rng, synth, h, w, minD, D, kind, seed):
    if kind == "noise":
        return (rng.integers(0, 256, (h, w), dtype=np.uint8), rng.integers(0, 256, (h, w), dtype=np.uint8))
    if kind == "binary":        # 0/255 noise against its (partly) negated copy: maximal costs
        left = (rng.integers(0, 2, (h, w)) * 255).astype(np.uint8)
        right = np.where(rng.random((h, w)) < 0.8, 255 - left, left).astype(np.uint8)
        return left, right
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=seed, with_truth=False)
    if kind == "flat":
        left, right = left.copy(), right.copy()
        for _ in range(int(rng.integers(1, 4))):
            y0, x0 = int(rng.integers(0, h)), int(rng.integers(0, w))
            hh, ww = int(rng.integers(1, h + 1)), int(rng.integers(1, w + 1))
            v = int(rng.integers(0, 256))
            left[y0:y0 + hh, x0:x0 + ww] = v
            right[y0:y0 + hh, max(x0 - 3, 0):x0 + ww] = v
    return left, right


def _case(pkg, seed):
    rng = np.random.default_rng(10_000 + seed)
    mode = [pkg.MODE_CENSUS8, pkg.MODE_OCV_SGBM5, pkg.MODE_OCV_HH8][seed % 3]
    D = int(rng.choice([16, 32, 48, 64, 80, 96, 128, 144, 256, 272, 400, 512]))
    minD = int(rng.integers(-12, 13))
    span = max(D + minD, 0)
    h = int(rng.choice([1, 2, 3, 7, 16, 23, 40]))
    w = span + int(rng.integers(1, 90)) if rng.random() < 0.85 else int(rng.integers(1, span + 4))
    kw = dict(num_disparities=D, min_disparity=minD,
              uniqueness_ratio=int(rng.choice([0, 1, 5, 10, 15, 30, 99, 100, 120])),
              disp12_max_diff=int(rng.choice([-1, 0, 1, 2, 5])),
              speckle_window_size=int(rng.choice([0, 0, 10, 50])), speckle_range=int(rng.integers(1, 4)))
    if mode == pkg.MODE_CENSUS8:
        p1 = int(rng.integers(1, 40))
        kw.update(p1=p1, p2=int(rng.integers(p1 + 1, 260)), subpixel=int(rng.integers(0, 2)),
                  lr_check=int(rng.integers(0, 2)), median=int(rng.integers(0, 2)))
    else:
        p1 = int(rng.integers(1, 300))
        kw.update(p1=p1, p2=int(rng.integers(p1 + 1, 1200)), block_size=int(rng.choice([1, 3, 5, 7, 9, 11, 15, 21])),
                  prefilter_cap=int(rng.integers(1, 64)))
    kind = str(rng.choice(["pair", "pair", "noise", "flat"]))
    if mode != pkg.MODE_CENSUS8:
        kw["ocv_compat"] = int(rng.integers(0, 8))
        if rng.random() < 0.2:
            kind = "binary"
            kw.update(block_size=int(rng.choice([15, 21, 31])), prefilter_cap=int(rng.integers(40, 64)),
                      p2=int(rng.integers(kw["p1"] + 1, 6000)))
    return rng, mode, h, w, kw, kind


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_match(engine, oracle, synth, pkg, seed):
    rng, mode, h, w, kw, kind = _case(pkg, seed)
    p = pkg.default_params(mode, **kw)
    engine.set_params(p)
    left, right = _images(rng, synth, h, w, kw["min_disparity"], kw["num_disparities"], kind, seed)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    env = {k: os.environ.get(k) for k in ("SGM_OCV_NO_BUF", "SGM_OCV_VWTA")}
    assert np.array_equal(got, ref), f"mode {mode} {h}x{w} {kw} {kind} {env}: {(got != ref).sum()} pixels differ"


def _ocv_fusable(h, w, kw):
    """ocv_cost_fusable() of csrc/ocv_sgm.hip without its size default (forced below)."""
    ftzero = max(kw["prefilter_cap"], 15) | 1
    block, minD, D = kw["block_size"], kw["min_disparity"], kw["num_disparities"]
    width1 = (w + min(minD, 0)) - max(minD + D, 0)
    return block // 2 <= 10 and block * block * (2 * ftzero + 63) <= 65535 and width1 > 0


@pytest.mark.parametrize("seed", [s for s in range(N_CASES) if s % 3])   # the OpenCV-mode cases
def test_fuzz_ocv_fused_cost(engine, oracle, synth, pkg, monkeypatch, seed):
    """Every OpenCV-mode case of test_fuzz_match again with the fused cost kernel forced
    (SGM_OCV_FUSED=1; the default only on frames of >= 10^8 cells) at a drawn disparity-pair
    block width (SGM_FUSE_DPC 8 / 16 / 32, falling back as the launcher does) and band height
    (SGM_FUSE_ROWS). Cases the kernel cannot take (boxes above 21, u16 box sums that could
    wrap, no valid column) run the unfused kernels and still must match."""
    rng, mode, h, w, kw, kind = _case(pkg, seed)
    sub = np.random.default_rng(70_000 + seed)
    monkeypatch.setenv("SGM_OCV_FUSED", "1")
    monkeypatch.setenv("SGM_FUSE_DPC", str(int(sub.choice([8, 16, 32]))))
    if sub.random() < 0.5:
        monkeypatch.setenv("SGM_FUSE_ROWS", str(int(sub.choice([1, 3, 16, 64]))))
    p = pkg.default_params(mode, **kw)
    engine.set_params(p)
    left, right = _images(rng, synth, h, w, kw["min_disparity"], kw["num_disparities"], kind, seed)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    tag = "fused" if _ocv_fusable(h, w, kw) else "unfused"
    assert np.array_equal(got, ref), f"[{tag}] mode {mode} {h}x{w} {kw} {kind}: {(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("seed", range(0, N_CASES, 3))        # the census cases
def test_fuzz_device_batch(engine, oracle, synth, pkg, seed):
    torch = pytest.importorskip("torch")
    rng, mode, h, w, kw, kind = _case(pkg, seed)
    assert mode == pkg.MODE_CENSUS8
    p = pkg.default_params(mode, **kw)
    engine.set_params(p)
    n = int(rng.integers(1, 6))
    frames = [_images(rng, synth, h, w, kw["min_disparity"], kw["num_disparities"], kind, seed + 97 * i)
              for i in range(n)]
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
    for i, (l, r) in enumerate(frames):
        ref = oracle.match(op, l, r)
        assert np.array_equal(got[i], ref), f"frame {i} of {n}, {h}x{w} {kw} {kind}: {(got[i] != ref).sum()} differ"


@pytest.mark.parametrize("seed", range(0, N_CASES, 3))        # the census cases
def test_fuzz_tiled_exact(engine, oracle, synth, pkg, seed):
    rng, mode, h, w, kw, kind = _case(pkg, seed)
    p = pkg.default_params(mode, **kw)
    engine.set_params(p)
    left, right = _images(rng, synth, h, w, kw["min_disparity"], kw["num_disparities"], kind, seed)
    bands = int(rng.integers(1, min(h, 6) + 1))
    got = engine.match_tiled_exact(left, right, bands)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{bands} bands, {h}x{w} {kw} {kind}: {(got != ref).sum()} pixels differ"


@pytest.mark.parametrize("seed", range(max(N_CASES // 2, 1)))
def test_fuzz_post_filters(engine, oracle, seed):
    """medianBlur(3) and filterSpeckles on random disparity images: piecewise-constant
    blobs, ramps and noise of random sizes, newVal / maxSize / maxDiff drawn at random."""
    rng = np.random.default_rng(50_000 + seed)
    h, w = int(rng.integers(1, 150)), int(rng.integers(1, 300))
    kind = int(rng.integers(0, 3))
    if kind == 0:       # blobs: a coarse random grid upsampled, plus sparse noise
        cy, cx = max(h // int(rng.integers(1, 12)), 1), max(w // int(rng.integers(1, 12)), 1)
        coarse = rng.integers(-40, 400, (h // cy + 1, w // cx + 1))
        disp = np.repeat(np.repeat(coarse, cy, 0), cx, 1)[:h, :w]
        m = rng.random((h, w)) < 0.05
        disp = np.where(m, rng.integers(-40, 400, (h, w)), disp)
    elif kind == 1:     # ramps: neighbours differ by small steps
        disp = (np.add.outer(np.arange(h) * int(rng.integers(0, 4)), np.arange(w) * int(rng.integers(0, 4))) % 500) - 20
    else:
        disp = rng.integers(-40, 400, (h, w))
    disp = disp.astype(np.int16)
    new_val = int(rng.choice([-16, -32, 0, int(disp.min())]))
    max_size, max_diff = int(rng.choice([0, 1, 5, 30, 100, 1000])), int(rng.choice([0, 1, 16, 32, 64]))
    assert np.array_equal(engine.median3(disp), oracle.median3(disp))
    got = engine.filter_speckles(disp, new_val, max_size, max_diff)
    ref = oracle.filter_speckles(disp, new_val, max_size, max_diff)
    assert np.array_equal(got, ref), f"{h}x{w} kind {kind} new {new_val} size {max_size} diff {max_diff}"


@pytest.mark.parametrize("seed", range(max(N_CASES // 4, 1)))
def test_fuzz_rectify(engine, oracle, seed):
    """initUndistortRectifyMap + INTER_CUBIC remap with random intrinsics, distortion models
    (0/4/5/8/12 coefficients), rotations and sizes: float32 maps and u8 output bit-exact."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(70_000 + seed)
    w, h = int(rng.integers(2, 400)), int(rng.integers(2, 300))
    f = float(rng.uniform(0.3, 2.0)) * w
    K = np.array([[f, 0, w / 2 + rng.normal(0, 5)], [0, f * rng.uniform(0.95, 1.05), h / 2 + rng.normal(0, 5)],
                  [0, 0, 1]], np.float64)
    nd = int(rng.choice([0, 4, 5, 8, 12]))
    Dd = rng.normal(0, 0.05, nd) * np.array([1, 0.5, 0.02, 0.02, 0.2, 0.2, 0.1, 0.1, 0.01, 0.01, 0.01, 0.01])[:nd]
    a = rng.normal(0, 0.05, 3)
    th = np.linalg.norm(a)
    k = a / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    P = np.array([[f * rng.uniform(0.8, 1.1), 0, w / 2 + rng.normal(0, 8), -0.1 * f],
                  [0, f * rng.uniform(0.8, 1.1), h / 2 + rng.normal(0, 8), 0], [0, 0, 1, 0]], np.float64)
    mx = torch.empty((h, w), dtype=torch.float32, device="cuda")
    my = torch.empty((h, w), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    engine.rectify_map(K, Dd, R, P, w, h, mx.data_ptr(), my.data_ptr(), w)
    engine.synchronize()
    rx, ry = oracle.rectify_map(K, Dd, R, P, w, h)
    assert np.array_equal(mx.cpu().numpy().view(np.uint32), rx.view(np.uint32)), "map x"
    assert np.array_equal(my.cpu().numpy().view(np.uint32), ry.view(np.uint32)), "map y"
    src = rng.integers(0, 256, (h, w), dtype=np.uint8)
    ds = torch.from_numpy(src).cuda()
    out = torch.empty((h, w), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    engine.remap_cubic(ds.data_ptr(), w, w, h, mx.data_ptr(), my.data_ptr(), w, w, h, out.data_ptr(), w)
    engine.synchronize()
    assert np.array_equal(out.cpu().numpy(), oracle.remap_cubic(src, rx, ry)), "remap"


@pytest.mark.parametrize("seed", range(max(N_CASES // 4, 1)))
def test_fuzz_depth(engine, oracle, pkg, seed):
    """DisparityImage packing and disparity -> depth / point cloud with random calibrations,
    depth windows, colour channels and disparity images (float32 bit-exact)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(90_000 + seed)
    h, w = int(rng.integers(1, 120)), int(rng.integers(1, 300))
    f = float(rng.uniform(200, 2000))
    cx, cy = w / 2 + rng.normal(0, 10), h / 2 + rng.normal(0, 10)
    K = np.array([[f, 0, cx], [0, f, cy], [0, 0, 1]])
    Pl = np.array([[f, 0, cx, 0], [0, f, cy, 0], [0, 0, 1, 0]])
    Pr = Pl.copy()
    Pr[0, 3] = -f * float(rng.uniform(0.03, 0.5))
    Pr[0, 2] = cx + rng.normal(0, 3)
    Q = oracle.calc_q(K, Pr, Pl)
    d = (rng.integers(-40, 4000, (h, w)) / 16.0).astype(np.float32)
    d[rng.random((h, w)) < 0.15] = 0
    d[rng.random((h, w)) < 0.1] = 10000
    lo = float(rng.choice([0.0, 0.1, 0.5]))
    window = (lo, lo + float(rng.choice([0.5, 3.0, 50.0, 1e4])))
    channels = int(rng.choice([0, 1, 3]))
    color = None if channels == 0 else rng.integers(0, 256, (h, w) if channels == 1 else (h, w, 3), dtype=np.uint8)
    depth, pts, rgba = pkg.disp_info_to_depth(engine, d, color, Q, *window)
    rd, rp, rr = oracle.depth_points(d, Q, *window, color)
    assert np.array_equal(depth.view(np.uint32), rd.view(np.uint32)), "depth"
    assert np.array_equal(pts.view(np.uint32), rp.view(np.uint32)), f"{len(pts)} vs {len(rp)} points"
    assert np.array_equal(rgba, rr), "colour"
    d16 = rng.integers(-300, 4000, (h, w)).astype(np.int16)
    src = torch.as_tensor(d16).cuda()
    out = torch.empty((h, w), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    engine.disparity_to_msg(src.data_ptr(), w, w, h, window[0], window[1], out.data_ptr(), w)
    engine.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle.disparity_to_msg(d16, *window).view(np.uint32))


@pytest.mark.parametrize("seed", range(max(N_CASES // 8, 1)))
def test_fuzz_fused_rectify_batch(engine, oracle, synth, pkg, seed):
    """Raw frames rectified inside the census tiles (sgm_match_device_batch_rect) with random
    raw / rectified sizes, calibrations, census parameters and frame counts: rectified images
    and disparities equal the oracle's remap and match of them."""
    torch = pytest.importorskip("torch")
    from test_rectify_oracle import calib
    rng = np.random.default_rng(110_000 + seed)
    D = int(rng.choice([16, 32, 64, 128]))
    minD = int(rng.integers(0, 8))
    rh, rw = int(rng.integers(8, 120)), int(rng.integers(D + minD + 8, D + minD + 200))
    h, w = max(int(rh * rng.uniform(0.8, 1.1)), 1), max(int(rw * rng.uniform(0.9, 1.1)), D + minD + 1)
    KL, DL, RL, PL = calib(seed=int(rng.integers(0, 1000)), w=rw, h=rh)
    KR, DR, RR, PR = calib(seed=int(rng.integers(0, 1000)), w=rw, h=rh)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, min_disparity=minD, p1=int(rng.integers(2, 20)),
                           p2=int(rng.integers(30, 190)), uniqueness_ratio=int(rng.choice([0, 5, 15])),
                           subpixel=int(rng.integers(0, 2)), lr_check=int(rng.integers(0, 2)),
                           median=int(rng.integers(0, 2)))
    engine.set_params(p)
    maps = []
    for K_, D_, R_, P_ in ((KL, DL, RL, PL), (KR, DR, RR, PR)):
        mx = torch.empty((h, w), dtype=torch.float32, device="cuda")
        my = torch.empty((h, w), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        engine.rectify_map(K_, D_, R_, P_, w, h, mx.data_ptr(), my.data_ptr(), w)
        engine.synchronize()
        maps.append((mx, my))
    n = int(rng.integers(1, 5))
    frames = [synth.stereo_pair(rh, rw, minD, D, seed=seed * 7 + i, with_truth=False)[:2] for i in range(n)]
    dl = [torch.as_tensor(f[0]).cuda() for f in frames]
    dr = [torch.as_tensor(f[1]).cuda() for f in frames]
    out = torch.full((n, h, w), 777, dtype=torch.int16, device="cuda")
    recl = torch.zeros((n, h, w), dtype=torch.uint8, device="cuda")
    recr = torch.zeros((n, h, w), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    engine.set_rectification((maps[0][0].data_ptr(), maps[0][1].data_ptr()),
                             (maps[1][0].data_ptr(), maps[1][1].data_ptr()), w, rw, rh)
    try:
        engine.match_device_batch_rect([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], w, h, rw,
                                       [recl[i].data_ptr() for i in range(n)], [recr[i].data_ptr() for i in range(n)],
                                       w, [out[i].data_ptr() for i in range(n)], w)
        engine.synchronize()
    finally:
        engine.set_rectification()
    rxl, ryl = oracle.rectify_map(KL, DL, RL, PL, w, h)
    rxr, ryr = oracle.rectify_map(KR, DR, RR, PR, w, h)
    op = to_oracle_params(oracle, p)
    got, gl, gr = out.cpu().numpy(), recl.cpu().numpy(), recr.cpu().numpy()
    for i, (l_raw, r_raw) in enumerate(frames):
        el, er = oracle.remap_cubic(l_raw, rxl, ryl), oracle.remap_cubic(r_raw, rxr, ryr)
        assert np.array_equal(gl[i], el) and np.array_equal(gr[i], er), f"frame {i} rectified"
        assert np.array_equal(got[i], oracle.match(op, el, er)), f"frame {i} of {n} disparity"


@pytest.mark.parametrize("seed", range(max(N_CASES // 4, 1)))
def test_fuzz_host_batch_and_overlap_tiles(engine, oracle, synth, pkg, seed):
    """Every mode through sgm_match_batch (host buffers, a thread + stream per device; the
    device list repeats device 0 to exercise the per-device workers) and, with a halo that
    covers the whole frame, through the overlap tile mode, which is then exact."""
    rng, mode, h, w, kw, kind = _case(pkg, 7000 + seed)
    p = pkg.default_params(mode, **kw)
    engine.set_params(p)
    n = int(rng.integers(1, 5))
    frames = [_images(rng, synth, h, w, kw["min_disparity"], kw["num_disparities"], kind, seed + 31 * i)
              for i in range(n)]
    outs = engine.match_batch([f[0] for f in frames], [f[1] for f in frames], devices=[0] * int(rng.integers(1, 3)))
    op = to_oracle_params(oracle, p)
    refs = [oracle.match(op, l, r) for l, r in frames]
    for i in range(n):
        assert np.array_equal(outs[i], refs[i]), f"batch frame {i} of {n}, mode {mode} {h}x{w} {kw} {kind}"
    bands = int(rng.integers(1, min(h, 4) + 1))
    got = engine.match_tiled(frames[0][0], frames[0][1], bands, h)
    assert np.array_equal(got, refs[0]), f"overlap tiles, {bands} bands, halo {h}, mode {mode} {h}x{w} {kw} {kind}"


@pytest.mark.parametrize("seed", range(max(N_CASES // 4, 8)))
def test_fuzz_ocv_large_disparity(engine, oracle, synth, pkg, monkeypatch, seed):
    """OpenCV modes with D > 512 (64-lane path lines, chunked one-pixel-per-wave WTA): random
    windows up to the cfg's 2048, blocks, penalties, uniqueness and post filters; half the cases
    with the step-rebased path descriptors forced (SGM_OCV_NO_BUF=1: the form of volumes past
    4 GB) and half with the fused vertical WTA forced (its deficit records for D <= 1024)."""
    rng = np.random.default_rng(50_000 + seed)
    sub = np.random.default_rng(70_000 + seed)          # the switches, apart from the case draws
    if sub.random() < 0.5:
        monkeypatch.setenv("SGM_OCV_NO_BUF", "1")
    if sub.random() < 0.5:
        monkeypatch.setenv("SGM_OCV_VWTA", "1")
    mode = [pkg.MODE_OCV_SGBM5, pkg.MODE_OCV_HH8][seed % 2]
    D = int(rng.choice([528, 640, 768, 1024, 1296, 1536, 2048]))
    minD = int(rng.integers(-12, 13))
    span = max(D + minD, 0)
    h = int(rng.choice([1, 3, 7, 16, 23]))
    w = span + int(rng.integers(1, 60)) if rng.random() < 0.9 else int(rng.integers(1, span + 4))
    p1 = int(rng.integers(1, 300))
    kw = dict(num_disparities=D, min_disparity=minD, p1=p1, p2=int(rng.integers(p1 + 1, 1200)),
              block_size=int(rng.choice([1, 3, 5, 7, 9, 11, 15, 21])), prefilter_cap=int(rng.integers(1, 64)),
              uniqueness_ratio=int(rng.choice([0, 1, 5, 10, 15, 30, 99, 100, 120])),
              disp12_max_diff=int(rng.choice([-1, 0, 1, 2, 5])),
              speckle_window_size=int(rng.choice([0, 0, 10, 50])), speckle_range=int(rng.integers(1, 4)))
    kind = str(rng.choice(["pair", "pair", "noise", "flat"]))
    p = pkg.default_params(mode, **kw)
    engine.set_params(p)
    left, right = _images(rng, synth, h, w, minD, min(D, 256), kind, seed)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    env = {k: os.environ.get(k) for k in ("SGM_OCV_NO_BUF", "SGM_OCV_VWTA")}
    assert np.array_equal(got, ref), f"mode {mode} {h}x{w} {kw} {kind} {env}: {(got != ref).sum()} pixels differ"
