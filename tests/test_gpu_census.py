"""GPU parity — census-SGM (north-star mode). Every comparison is bit-exact (int16/u8/u64).

Stage by stage against the CPU oracle: census codes, each of the 7 stored path volumes,
then the full pipeline (dir 7 + 8-way sum + WTA + uniqueness + subpixel + LR), post
filters, golden fixtures, and the BASELINE sizes (1920x1080 D=128 / D=256).
"""
import numpy as np
import pytest

from conftest import to_oracle_params

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(1, 1), (5, 7), (48, 64), (37, 101), (72, 300)])
def test_census_codes(engine, oracle, shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    img[::3, ::2] = 77
    assert np.array_equal(engine.census(img), oracle.census(img))


@pytest.mark.parametrize("D,minD", [(16, 0), (32, -7), (64, 3), (128, 0), (256, 0), (512, 0), (48, 2), (80, -3),
                                    (272, 0), (400, -5)])
@pytest.mark.parametrize("dirn", range(8))
def test_census_path_volumes(engine, oracle, synth, pkg, dirn, D, minD):
    h = 23
    w = max(D + minD, 0) + 57
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=D + dirn)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, min_disparity=minD, p1=9, p2=110)
    engine.set_params(p)
    got = engine.census_path(left, right, dirn)
    ref = oracle.census_path(to_oracle_params(oracle, p), left, right, dirn)
    assert np.array_equal(got, ref), f"dir {dirn}: {(got != ref).sum()} cells differ"


CASES = [
    dict(num_disparities=64),
    dict(num_disparities=64, subpixel=0),
    dict(num_disparities=64, lr_check=0),
    dict(num_disparities=32, min_disparity=5, uniqueness_ratio=15),
    dict(num_disparities=32, min_disparity=-9),
    dict(num_disparities=16, p1=3, p2=20, disp12_max_diff=3),
    dict(num_disparities=128, median=1),
    dict(num_disparities=96, speckle_window_size=30, speckle_range=2, median=1),
    dict(num_disparities=256, uniqueness_ratio=0),
    dict(num_disparities=512),
    dict(num_disparities=64, p2=250),         # clamped to 193 (u8 path costs)
    dict(num_disparities=400, min_disparity=3),   # D % 32 == 16: a lane straddles D (DPL 32)
    dict(num_disparities=64, uniqueness_ratio=99),
    dict(num_disparities=64, uniqueness_ratio=100),   # every d qualifies when minS > 0
    dict(num_disparities=48, uniqueness_ratio=130),   # > 100: S > 0 qualifies when minS == 0
    dict(num_disparities=32, uniqueness_ratio=1, p2=15),
]


@pytest.mark.parametrize("kw", CASES, ids=[str(i) for i in range(len(CASES))])
def test_census_pipeline(engine, oracle, synth, pkg, kw):
    D, minD = kw["num_disparities"], kw.get("min_disparity", 0)
    h, w = 61, max(D + minD, 0) + 133
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=D + 17)
    p = pkg.default_params(pkg.MODE_CENSUS8, **kw)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


def test_census_edge_geometry(engine, oracle, pkg):
    rng = np.random.default_rng(3)
    for (h, w, D, minD) in [(4, 20, 16, 0), (3, 17, 16, 0), (9, 16, 16, 0), (30, 40, 48, 0), (2, 200, 64, -30)]:
        left = rng.integers(0, 256, (h, w), dtype=np.uint8)
        right = rng.integers(0, 256, (h, w), dtype=np.uint8)
        p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, min_disparity=minD, median=1)
        engine.set_params(p)
        assert np.array_equal(engine.match(left, right), oracle.match(to_oracle_params(oracle, p), left, right))


def test_census_strided_host_buffers(engine, oracle, synth, pkg):
    left, right, _ = synth.stereo_pair(40, 150, 0, 32, seed=4)
    big_l = np.zeros((40, 160), np.uint8)
    big_r = np.zeros((40, 160), np.uint8)
    big_l[:, :150], big_r[:, :150] = left, right
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=32)
    engine.set_params(p)
    out = np.full((40, 170), 1234, np.int16)
    import ctypes
    rc = engine.lib.sgm_match(engine.h, ctypes.c_void_p(big_l.ctypes.data), ctypes.c_void_p(big_r.ctypes.data),
                              150, 40, 160, ctypes.c_void_p(out.ctypes.data), 170)
    assert rc == 0
    assert np.array_equal(out[:, :150], oracle.match(to_oracle_params(oracle, p), left, right))
    assert (out[:, 150:] == 1234).all()


def test_bad_params_fail_at_match_time(engine, pkg):
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=40)
    engine.set_params(p)                     # setters never fail (reference behaviour)
    z = np.zeros((16, 64), np.uint8)
    with pytest.raises(pkg.SGMError) as e:
        engine.match(z, z)
    assert e.value.code == pkg.SGM_ERR_PARAM and "16" in str(e.value)


def test_golden_fixtures(engine, oracle, pkg):
    import os
    gdir = os.path.join(os.path.dirname(__file__), "golden")
    n = 0
    for f in sorted(os.listdir(gdir)):
        if not f.endswith(".npz"):
            continue
        z = np.load(os.path.join(gdir, f), allow_pickle=False)
        p = pkg.SgmParams()
        for k, v in zip(z["param_names"], z["param_values"]):
            setattr(p, str(k), int(v))
        engine.set_params(p)
        got = engine.match(z["left"], z["right"])
        assert np.array_equal(got, z["disp"]), f"{f}: {(got != z['disp']).sum()} pixels differ"
        n += 1
    assert n >= 8


@pytest.mark.parametrize("D", [128, 256])
def test_full_size_baseline_configs(engine, oracle, synth, pkg, D):
    """BASELINE configs C2 (D=128, no subpix/LR) and C3 (D=256 + subpix + LR) at 1920x1080,
    bit-exact against the oracle (multi-threaded CPU, a few seconds on the box)."""
    left, right, _ = synth.stereo_pair(1080, 1920, 0, D, seed=D)
    kw = dict(num_disparities=D, p1=10, p2=120, uniqueness_ratio=5)
    if D == 128:
        kw.update(subpixel=0, lr_check=0)
    p = pkg.default_params(pkg.MODE_CENSUS8, **kw)
    engine.set_params(p)
    got = engine.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
    # size-independent sanity: accuracy vs the synthetic truth
    _, _, g = synth.stereo_pair(1080, 1920, 0, D, seed=D)
    m = got != -16
    assert m.mean() > 0.6 and np.median(np.abs(got[m] / 16.0 - g[m])) < 0.6


def test_repeat_and_resize(engine, oracle, synth, pkg):
    """Workspace reuse across frames and geometry/parameter changes between frames."""
    for (h, w, D) in [(40, 120, 32), (64, 200, 64), (40, 120, 32), (30, 90, 16)]:
        left, right, _ = synth.stereo_pair(h, w, 0, D, seed=h + w)
        p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D)
        engine.set_params(p)
        a = engine.match(left, right)
        b = engine.match(left, right)
        assert np.array_equal(a, b)
        assert np.array_equal(a, oracle.match(to_oracle_params(oracle, p), left, right))


def test_batch_equals_single(engine, pkg, synth):
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=64)
    engine.set_params(p)
    frames = [synth.stereo_pair(48, 160, 0, 64, seed=100 + i) for i in range(5)]
    outs = engine.match_batch([f[0] for f in frames], [f[1] for f in frames])
    for (l, r, _), o in zip(frames, outs):
        assert np.array_equal(o, engine.match(l, r))


def test_device_pointer_path(engine, pkg, synth):
    torch = pytest.importorskip("torch")
    left, right, _ = synth.stereo_pair(64, 256, 0, 64, seed=9)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=64)
    engine.set_params(p)
    ref = engine.match(left, right)
    dl = torch.from_numpy(left).cuda()
    dr = torch.from_numpy(right).cuda()
    out = torch.empty((64, 256), dtype=torch.int16, device="cuda")
    stream = torch.cuda.Stream()                 # explicit non-default stream handed to the C-ABI
    stream.wait_stream(torch.cuda.current_stream())
    engine.match_device(dl.data_ptr(), dr.data_ptr(), 256, 64, 256, out.data_ptr(), 256, stream.cuda_stream)
    stream.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)


def test_profiling_stage_times(engine, pkg, synth):
    left, right, _ = synth.stereo_pair(64, 256, 0, 64, seed=9)
    engine.set_params(pkg.default_params(pkg.MODE_CENSUS8, num_disparities=64))
    engine.set_profiling(True)
    engine.match(left, right)
    st = engine.stage_times()
    engine.set_profiling(False)
    names = [s[0] for s in st]
    assert names[:3] == ["census", "paths8", "wta_lr"]
    assert all(t >= 0 for _, t, _ in st) and all(b > 0 for _, _, b in st)


@pytest.mark.parametrize("up_wta", [1, 0])
@pytest.mark.parametrize("kw,n", [(dict(num_disparities=64), 2), (dict(num_disparities=48, min_disparity=3), 3),
                                  (dict(num_disparities=128, median=1, speckle_window_size=20, speckle_range=2), 4),
                                  (dict(num_disparities=256), 5), (dict(num_disparities=32), 1),
                                  (dict(num_disparities=400, median=1), 7)])
def test_device_batch_pipeline(engine, oracle, pkg, synth, monkeypatch, kw, n, up_wta):
    """sgm_match_device_batch (the sweeps of one group of frames fused with the WTA of the
    previous group) returns exactly the per-frame results, for every frame of the batch, in
    both schemes: the up+WTA one (the previous group's upward sweep carries its WTA, so its
    volume is never stored) and the earlier one (SGM_UPWTA=0: eight volumes, WTA rows)."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("SGM_UPWTA", str(up_wta))
    D, minD = kw["num_disparities"], kw.get("min_disparity", 0)
    h, w = 45, max(D + minD, 0) + 150
    p = pkg.default_params(pkg.MODE_CENSUS8, **kw)
    engine.set_params(p)
    frames = [synth.stereo_pair(h, w, max(minD, 0), D, seed=300 + 7 * i + D) for i in range(n)]
    dl = [torch.from_numpy(f[0]).cuda() for f in frames]
    dr = [torch.from_numpy(f[1]).cuda() for f in frames]
    out = torch.full((n, h, w), 777, dtype=torch.int16, device="cuda")
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    engine.set_profiling(True)
    engine.match_device_batch([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], w, h, w,
                              [out[i].data_ptr() for i in range(n)], w, stream.cuda_stream)
    stream.synchronize()
    launches = engine.stage_launches()
    engine.set_profiling(False)
    got = out.cpu().numpy()
    op = to_oracle_params(oracle, p)
    for i, (l, r, _) in enumerate(frames):
        ref = oracle.match(op, l, r)
        assert np.array_equal(got[i], ref), f"frame {i}: {(got[i] != ref).sum()} pixels differ"
    ng = (n + 1) // 2         # groups of (default) 2 frames
    assert launches["census"] == min(n, 2)
    if n == 1:                # one frame: the single-frame pipeline (no group to fuse with)
        assert launches["paths8"] == 1 and launches["wta_lr"] == 1
    elif up_wta and D <= 256:
        # census(G0) | fused[paths7(G0) + census(G1)] | fused[paths7(Gk) + upWTA(Gk-1) + census(Gk+1)]
        # rowfin ... | fused[paths8(Glast) + upWTA(Glast-1)] rowfin | wta(Glast)
        assert launches["wta_lr"] == 1 and launches.get("rowfin", 0) == ng - 1
        if ng == 1:
            assert launches["paths8"] == 1
        else:
            assert launches["paths7+census"] == 1 and launches["paths8+up_wta"] == 1
            assert launches.get("paths7+up_wta+census", 0) == ng - 2
    else:
        # census(G0) | fused[paths(G0) + census(G1)] | fused[paths(Gk) + wta(Gk-1) + census(Gk+1)]
        # ... | fused[paths(Glast) + wta] | wta(Glast)
        assert launches["wta_lr"] == 1
        if ng == 1:
            assert launches["paths8"] == 1
        else:
            assert launches["paths8+census"] == 1 and launches["paths8+wta_lr"] == 1
            assert launches.get("paths8+wta_lr+census", 0) == ng - 2


def test_tiled_single_band_is_exact(engine, oracle, synth, pkg):
    """sgm_match_tiled with one band is the full-frame match."""
    left, right, _ = synth.stereo_pair(96, 256, 0, 64, seed=41)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=64)
    engine.set_params(p)
    assert np.array_equal(engine.match_tiled(left, right, 1, 0), oracle.match(to_oracle_params(oracle, p), left, right))


@pytest.mark.parametrize("bands,halo", [(4, 0), (4, 16), (4, 64), (8, 128)])
def test_tiled_overlap_mode_disagreement(engine, oracle, synth, pkg, bands, halo):
    """SURVEY §8(e) C5 overlap mode: row bands with halos, no path-state exchange. Each band
    equals the oracle run on its extended rows (exact), and the disagreement with the
    full-frame result shrinks as the halo grows (reported)."""
    h, w, D = 384, 448, 128
    left, right, _ = synth.stereo_pair(h, w, 0, D, seed=43)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D)
    engine.set_params(p)
    got = engine.match_tiled(left, right, bands, halo)
    op = to_oracle_params(oracle, p)
    for b in range(bands):
        c0, c1 = b * h // bands, (b + 1) * h // bands
        e0, e1 = max(0, c0 - halo), min(h, c1 + halo)
        ref = oracle.match(op, left[e0:e1], right[e0:e1])
        assert np.array_equal(got[c0:c1], ref[c0 - e0:c1 - e0]), f"band {b}"
    full = oracle.match(op, left, right)
    frac = float((got != full).mean())
    print(f"bands={bands} halo={halo}: {100 * frac:.3f} % of pixels differ from the full-frame match")
    assert frac < {0: 0.1, 16: 0.01, 64: 0.001, 128: 0.001}[halo]


@pytest.fixture(scope="module")
def c5_case(synth, pkg, oracle):
    """BASELINE config C5 (4096x3000, D=512, 8-path + subpixel + LR): the frame, its parameters
    and the oracle's disparity (OpenMP over lines; ~20 s and ~11 GB of host RAM for S), computed
    once for the C5 tests."""
    h, w, D = 3000, 4096, 512
    left, right, _ = synth.stereo_pair(h, w, 0, D, seed=5, with_truth=False)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    return left, right, p, ref


@pytest.mark.timeout(600)
def test_c5_full_frame_vs_oracle(engine, c5_case):
    """C5 on one device against the oracle, bit for bit: the 32-lane path lines,
    5.5 GB direction volumes (64-bit offsets: where a 32-bit overflow was once found) and the
    lone frame's WTA at full size."""
    left, right, p, ref = c5_case
    engine.set_params(p)
    got = engine.match(left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"
    assert (ref != -16).mean() > 0.5


def test_c5_tiled_vs_full_frame(engine, c5_case):
    """C5: 8 row bands with a 128-row halo (the 8-GPU layout, run here on the visible devices)
    against the full frame (the oracle's)."""
    left, right, p, full = c5_case
    engine.set_params(p)
    tiled = engine.match_tiled(left, right, 8, 128)
    frac = float((tiled != full).mean())
    print(f"C5 8 bands, halo 128: {100 * frac:.4f} % of pixels differ from the full frame")
    assert frac < 0.001
    assert (full != -16).mean() > 0.5


@pytest.mark.parametrize("bands,halo,n_dev,pad", [(1, 0, 1, 0), (3, 16, 2, 0), (4, 64, 4, 13), (5, 200, 3, 7),
                                                    (2, 32, 2, 9)])
def test_tiled_device_equals_host_tiles(engine, oracle, synth, pkg, bands, halo, n_dev, pad):
    """sgm_match_tiled_device (device buffers, band b on devices[b % n], here all device 0 as
    bench.py --config c5 runs it with N bands on one GPU) is band for band the oracle on the
    band's extended rows, i.e. the host overlap mode; strided input / output rows included (one
    2-D copy per band and direction, the call the cross-device bands make too)."""
    import torch
    h, w, D = 200, 320, 96
    left, right, _ = synth.stereo_pair(h, w, 0, D, seed=47 + bands)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, median=1, speckle_window_size=20, speckle_range=2)
    engine.set_params(p)
    s_in, s_out = w + pad, w + 2 * pad
    dl = torch.zeros((h, s_in), dtype=torch.uint8, device="cuda")
    dr = torch.zeros((h, s_in), dtype=torch.uint8, device="cuda")
    dl[:, :w] = torch.from_numpy(left).cuda()
    dr[:, :w] = torch.from_numpy(right).cuda()
    out = torch.full((h, s_out), 1234, dtype=torch.int16, device="cuda")
    engine.match_tiled_device(dl.data_ptr(), dr.data_ptr(), w, h, s_in, out.data_ptr(), s_out, bands, halo,
                              devices=[0] * n_dev)
    got = out.cpu().numpy()
    assert (got[:, w:] == 1234).all()                       # row padding untouched
    got = got[:, :w]
    assert np.array_equal(got, engine.match_tiled(left, right, bands, halo))
    op = to_oracle_params(oracle, p)
    for b in range(bands):
        c0, c1 = b * h // bands, (b + 1) * h // bands
        e0, e1 = max(0, c0 - halo), min(h, c1 + halo)
        assert np.array_equal(got[c0:c1], oracle.match(op, left[e0:e1], right[e0:e1])[c0 - e0:c1 - e0]), f"band {b}"


def test_bench_c5_block_on_one_device():
    """bench.py --config c5 --gpus 1 (the driver's default run adds the same block): the full
    frame on one device, with its roofline and stage split."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--config", "c5", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert res["n_gpus"] == 1 and res["c5"]["disagreement_vs_full_frame"] == 0.0
    assert 0.2 < res["roofline"]["frac"] < 1.0 and "paths8" in " ".join(res["c5"]["stages"])


EXACT_CASES = [
    (dict(num_disparities=64), 2),
    (dict(num_disparities=64), 5),
    (dict(num_disparities=48, min_disparity=2), 3),        # D < 16*DPL: masked lanes in the seed
    (dict(num_disparities=32, min_disparity=-9), 4),       # negative minD (maxX1 < W)
    (dict(num_disparities=128, median=1, speckle_window_size=30, speckle_range=2), 4),  # post on the frame
    (dict(num_disparities=256, uniqueness_ratio=0), 3),
    (dict(num_disparities=400, min_disparity=3), 2),       # DPL 32, lane straddling D
    (dict(num_disparities=64), 61),                        # one-row bands
]


@pytest.mark.parametrize("kw,bands", EXACT_CASES, ids=[str(i) for i in range(len(EXACT_CASES))])
def test_tiled_exact_equals_full_frame(engine, oracle, synth, pkg, kw, bands):
    """SURVEY §8(e) exact mode: path lines continue across band seams through the
    boundary-row exchange, so every band count gives the full-frame result bit for bit."""
    D, minD = kw["num_disparities"], kw.get("min_disparity", 0)
    h, w = 61, max(D + minD, 0) + 133
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=D + bands)
    p = pkg.default_params(pkg.MODE_CENSUS8, **kw)
    engine.set_params(p)
    got = engine.match_tiled_exact(left, right, bands)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} pixels differ"


def test_tiled_exact_band_devices_and_reuse(engine, oracle, synth, pkg):
    """Bands dealt over an explicit device list (all device 0 here, the 8-GPU layout of
    C5 on one card), the band handles reused across calls and geometry changes."""
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=64)
    engine.set_params(p)
    op = to_oracle_params(oracle, p)
    for (h, w, bands, seed) in [(96, 256, 8, 3), (40, 200, 3, 4), (96, 256, 8, 5)]:
        left, right, _ = synth.stereo_pair(h, w, 0, 64, seed=seed)
        got = engine.match_tiled_exact(left, right, bands, devices=[0] * 8)
        assert np.array_equal(got, oracle.match(op, left, right)), (h, w, bands)


def test_tiled_exact_no_disparity_window(engine, pkg):
    """width1 <= 0 (D wider than the image): every pixel invalid, as in sgm_match."""
    left = np.full((20, 40), 9, np.uint8)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=64)
    engine.set_params(p)
    got = engine.match_tiled_exact(left, left, 3)
    assert np.array_equal(got, engine.match(left, left))
    assert (got == -16).all()


def test_c5_tiled_exact_vs_full_frame(engine, c5_case):
    """BASELINE config C5 (4096x3000, D=512) in exact mode: 8 bands with boundary-row
    exchange equal the full frame (the oracle's) at every pixel."""
    left, right, p, full = c5_case
    engine.set_params(p)
    tiled = engine.match_tiled_exact(left, right, 8)
    assert np.array_equal(tiled, full), f"{(tiled != full).sum()} pixels differ"


@pytest.mark.parametrize("D", [64, 48])
@pytest.mark.parametrize("kw", [dict(), dict(speckle_window_size=30, speckle_range=2), dict(median=1)])
@pytest.mark.parametrize("f32", [False, True])
def test_registered_output_copy_out(engine, oracle, synth, pkg, kw, f32, D):
    """sgm_host_register'ed outputs (the adapter's persistent disparity_lr, page-locked and mapped):
    same result as the oracle and as an unregistered output, with and without post filters, in
    sgm_match (int16, copied back by DMA) and sgm_match_f32 (without post filters the WTA writes
    the float rows straight into the mapped buffer, k_census_wta16f), the registration reused
    across calls; the right image's copy overlaps the left census (second stream)."""
    h, w = 203, 300
    left, right, _ = synth.stereo_pair(h, w, 0, D, seed=77)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, **kw)
    engine.set_params(p)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    pad = 5
    buf = np.full((h, w + pad), -7, np.float32 if f32 else np.int16)
    out = buf[:, :w]
    engine.host_register(buf)
    try:
        for _ in range(2):                                  # the second call reuses the registration
            out[...] = -7
            if f32:
                engine.match_f32(left, right, out=out)
            else:
                engine._check(engine.lib.sgm_match(engine.h, left.ctypes.data, right.ctypes.data, w, h, w,
                                                   out.ctypes.data, buf.shape[1]))
            got = out.astype(np.float32) if f32 else out
            assert np.array_equal(got, ref.astype(got.dtype))
            assert (buf[:, w:] == -7).all()
    finally:
        engine.host_unregister(buf)
    plain = engine.match_f32(left, right) if f32 else engine.match(left, right)
    assert np.array_equal(plain, ref.astype(plain.dtype))
