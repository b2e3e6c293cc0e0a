"""Pins the CPU oracle (oracle/sgm_oracle.c) before it is trusted as the GPU checker.

The reference has no tests, fixtures or golden vectors and OpenCV is absent,
so the oracle is pinned by (a) analytic known-answer tests, (b) independent numpy
restatements of each stage written from the published algorithm, and (c) its own committed
golden fixtures (regression pin, tests/golden/make_golden.py). Parity against real OpenCV
stays **unpinned** (DESIGN.md §Parity).
"""
import os
from collections import deque

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


# ------------------------------------------------------------------ independent numpy restatements
def np_census(img):
    h, w = img.shape
    p = np.pad(img.astype(np.int32), ((3, 3), (4, 4)), mode="edge")
    c = img.astype(np.int32)
    code = np.zeros((h, w), np.uint64)
    bit = 0
    for dy in range(-3, 4):
        for dx in range(-4, 5):
            if dx == 0 and dy == 0:
                continue
            nb = p[3 + dy:3 + dy + h, 4 + dx:4 + dx + w]
            code |= (nb < c).astype(np.uint64) << np.uint64(bit)
            bit += 1
    return code


def np_popcount64(a):
    a = a.astype(np.uint64)
    cnt = np.zeros(a.shape, np.int32)
    for s in range(0, 64, 8):
        byte = ((a >> np.uint64(s)) & np.uint64(0xFF)).astype(np.int32)
        cnt += np.array([bin(i).count("1") for i in range(256)], np.int32)[byte]
    return cnt


def np_census_cost(cl, cr, minD, D):
    h, w = cl.shape
    minX1, maxX1 = max(minD + D, 0), w + min(minD, 0)
    C = np.zeros((h, maxX1 - minX1, D), np.int32)
    for k in range(D):
        xs = np.arange(minX1, maxX1)
        C[:, :, k] = np_popcount64(cl[:, xs] ^ cr[:, xs - minD - k])
    return C


def np_path(C, rx, ry, P1, P2, u8=True):
    """Direction-independent recurrence L(p) = C + min(Lp, Lp(d+-1)+P1, minLp+P2) - minLp."""
    H, W1, D = C.shape
    L = np.zeros_like(C)
    order_y = range(H) if ry >= 0 else range(H - 1, -1, -1)
    order_x = list(range(W1)) if rx >= 0 else list(range(W1 - 1, -1, -1))
    big = 1 << 20
    for y in order_y:
        for x in order_x:
            py, px = y - ry, x - rx
            if 0 <= py < H and 0 <= px < W1 and not (rx == 0 and ry == 0):
                lp = L[py, px]
                m = lp.min()
                lm1 = np.concatenate([[big], lp[:-1]])
                lp1 = np.concatenate([lp[1:], [big]])
                best = np.minimum(np.minimum(lp, np.minimum(lm1, lp1) + P1), m + P2)
                L[y, x] = C[y, x] + best - m
            else:
                L[y, x] = C[y, x]
    return L


def np_bt_cost(left, right, minD, D, ftzero):
    """calcPixelCostBT for all rows (mono) — written from the published algorithm."""
    h, w = left.shape

    def prefilter(img):
        i = img.astype(np.int32)
        n = np.vstack([i[:1], i[:-1]])
        s = np.vstack([i[1:], i[-1:]])
        pf = np.full((h, w), ftzero, np.int32)
        raw = np.full((h, w), ftzero, np.int32)
        v = (i[:, 2:] - i[:, :-2]) * 2 + n[:, 2:] - n[:, :-2] + s[:, 2:] - s[:, :-2]
        pf[:, 1:-1] = np.clip(v, -ftzero, ftzero) + ftzero
        raw[:, 1:-1] = i[:, 1:-1]
        return pf, raw

    def lohi(a):
        l = np.concatenate([a[:, :1], (a[:, 1:] + a[:, :-1]) // 2], axis=1)
        r = np.concatenate([(a[:, :-1] + a[:, 1:]) // 2, a[:, -1:]], axis=1)
        return np.minimum(np.minimum(l, r), a), np.maximum(np.maximum(l, r), a)

    minX1, maxX1 = max(minD + D, 0), w + min(minD, 0)
    cost = np.zeros((h, maxX1 - minX1, D), np.int32)
    for ch, shift in ((0, 0), (1, 2)):
        a1 = prefilter(left)[ch]
        a2 = prefilter(right)[ch]
        lo1, hi1 = lohi(a1)
        lo2, hi2 = lohi(a2)
        xs = np.arange(minX1, maxX1)
        for k in range(D):
            xr = xs - minD - k
            u, u0, u1 = a1[:, xs], lo1[:, xs], hi1[:, xs]
            v, v0, v1 = a2[:, xr], lo2[:, xr], hi2[:, xr]
            c0 = np.maximum(0, np.maximum(u - v1, v0 - u))
            c1 = np.maximum(0, np.maximum(v - u1, u0 - v))
            cost[:, :, k] += np.minimum(c0, c1) >> shift
    return cost


def np_box_cost(pix, SW2, SH2, P2, fullDP, col0_legacy=False):
    """Exact replicate box sum + OpenCV's bottom-row rule + P2 offset (+ the 3.x rule: column 0
    of rows y >= 1 keeps row 0's value, or P2 in MODE_HH)."""
    H, W1, D = pix.shape
    xi = np.clip(np.arange(W1)[:, None] + np.arange(-SW2, SW2 + 1)[None, :], 0, W1 - 1)
    hs = pix[:, xi, :].sum(axis=2)
    yi = np.clip(np.arange(H)[:, None] + np.arange(-SH2, SH2 + 1)[None, :], 0, H - 1)
    vs = hs[yi].sum(axis=1)
    C = P2 + vs
    last = max(H - 1 - SH2, 0)
    for y in range(1, H):
        if y + SH2 >= H:
            C[y] = P2 if fullDP else C[last]
    if col0_legacy:
        C[1:, 0] = P2 if fullDP else C[0, 0]
    return C


def np_median3(d):
    p = np.pad(d, 1, mode="edge")
    h, w = d.shape
    stack = np.stack([p[dy:dy + h, dx:dx + w] for dy in range(3) for dx in range(3)])
    return np.median(stack, axis=0).astype(np.int16)


def py_speckle(d, new_val, max_size, max_diff):
    d = d.copy()
    h, w = d.shape
    lab = -np.ones((h, w), np.int64)
    comps = []
    for y in range(h):
        for x in range(w):
            if d[y, x] == new_val or lab[y, x] >= 0:
                continue
            q = deque([(y, x)])
            lab[y, x] = len(comps)
            members = []
            while q:
                cy, cx = q.popleft()
                members.append((cy, cx))
                for ny, nx in ((cy + 1, cx), (cy - 1, cx), (cy, cx + 1), (cy, cx - 1)):
                    if 0 <= ny < h and 0 <= nx < w and lab[ny, nx] < 0 and d[ny, nx] != new_val \
                            and abs(int(d[cy, cx]) - int(d[ny, nx])) <= max_diff:
                        lab[ny, nx] = len(comps)
                        q.append((ny, nx))
            comps.append(members)
    for m in comps:
        if len(m) <= max_size:
            for (y, x) in m:
                d[y, x] = new_val
    return d


# ------------------------------------------------------------------ stage cross-checks
@pytest.mark.parametrize("shape", [(7, 9), (20, 33), (31, 64)])
def test_census_matches_numpy(oracle, shape):
    rng = np.random.default_rng(shape[0] * 100 + shape[1])
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    img[3:5, 2:6] = 128  # ties: "<" is strict
    assert np.array_equal(oracle.census(img), np_census(img))


@pytest.mark.parametrize("dirn", range(8))
@pytest.mark.parametrize("minD,D", [(0, 16), (-5, 32), (3, 16)])
def test_census_path_matches_numpy(oracle, synth, dirn, minD, D):
    left, right, _ = synth.stereo_pair(14, 60, max(minD, 0), D, seed=dirn + D)
    p = oracle.make_params(oracle.MODE_CENSUS8, min_disparity=minD, num_disparities=D, p1=7, p2=90)
    C = np_census_cost(oracle.census(left), oracle.census(right), minD, D)
    rx, ry = oracle.DIRS[dirn]
    ref = np_path(C, rx, ry, 7, 90)
    got = oracle.census_path(p, left, right, dirn)
    assert got.dtype == np.uint8 and ref.max() <= 255
    assert np.array_equal(got.astype(np.int32), ref)


@pytest.mark.parametrize("compat", [0, 1, 7])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("h,w,minD,D,block,cap", [(12, 50, 0, 16, 5, 31), (9, 45, 4, 16, 7, 15),
                                                  (4, 40, -3, 16, 9, 63), (17, 70, 2, 32, 3, 1)])
def test_ocv_cost_matches_numpy(oracle, mode, h, w, minD, D, block, cap, compat):
    """C' against a numpy box sum, for the scalar, 3.x-column-0 and melodic builds (no sum
    leaves int16 here, so the SIMD saturation cannot show)."""
    rng = np.random.default_rng(h * w + mode)
    left = rng.integers(0, 256, (h, w), dtype=np.uint8)
    right = rng.integers(0, 256, (h, w), dtype=np.uint8)
    p = oracle.make_params(mode, min_disparity=minD, num_disparities=D, block_size=block, prefilter_cap=cap,
                           p1=8, p2=32, ocv_compat=compat)
    e = oracle.effective(p, w, h)
    pix = np_bt_cost(left, right, minD, D, e["ftzero"])
    ref = np_box_cost(pix, e["SW2"], e["SH2"], e["P2"], mode == 1, bool(compat & 1))
    got = oracle.ocv_cost(p, left, right)
    assert np.array_equal(got.astype(np.int64), ref)


def test_median_matches_numpy(oracle):
    rng = np.random.default_rng(5)
    d = rng.integers(-300, 3000, (23, 37)).astype(np.int16)
    assert np.array_equal(oracle.median3(d), np_median3(d))


@pytest.mark.parametrize("max_size,max_diff", [(0, 16), (5, 16), (30, 64), (1000, 0)])
def test_speckles_match_bfs(oracle, max_size, max_diff):
    rng = np.random.default_rng(max_size + max_diff)
    d = (rng.integers(0, 6, (24, 31)) * 16).astype(np.int16)
    d[rng.random((24, 31)) < 0.15] = -16
    ref = py_speckle(d, -16, max_size, max_diff)
    assert np.array_equal(oracle.filter_speckles(d, -16, max_size, max_diff), ref)


def test_wta_matches_full_census_pipeline(oracle, synth):
    left, right, _ = synth.stereo_pair(30, 90, 0, 32, seed=3)
    p = oracle.make_params(oracle.MODE_CENSUS8, num_disparities=32, median=0)
    S = oracle.census_sum(p, left, right)
    assert np.array_equal(oracle.wta(p, S, 90), oracle.match(p, left, right))


# ------------------------------------------------------------------ known-answer tests
@pytest.mark.parametrize("shift", [3, 11, 25])
def test_kat_integer_shift_census(oracle, synth, shift):
    left, right = synth.integer_shift_pair(40, 120, shift, seed=shift)
    p = oracle.make_params(oracle.MODE_CENSUS8, num_disparities=32, subpixel=0, lr_check=1)
    d = oracle.match(p, left, right)
    e = oracle.effective(p, 120, 40)
    assert (d[:, :e["minX1"]] == e["invalid"]).all()      # columns < maxD are invalid
    inner = d[:, e["minX1"]:e["maxX1"]]
    assert (inner == shift * 16).mean() > 0.99


@pytest.mark.parametrize("mode", [0, 1])
def test_kat_integer_shift_ocv(oracle, synth, mode):
    left, right = synth.integer_shift_pair(40, 120, 9, seed=9)
    p = oracle.make_params(mode, min_disparity=0, num_disparities=32, block_size=5, speckle_window_size=0)
    d = oracle.match(p, left, right)
    inner = d[:, 32:]
    valid = inner != -16
    assert valid.mean() > 0.95
    assert (np.round(inner[valid] / 16.0) == 9).mean() > 0.99


def test_kat_slanted_plane_subpixel(oracle, synth):
    left, right, g = synth.stereo_pair(120, 200, 0, 64, seed=3)
    d = oracle.match(oracle.make_params(oracle.MODE_CENSUS8, num_disparities=64), left, right)
    m = d != -16
    err = np.abs(d[m] / 16.0 - g[m])
    assert np.median(err) < 0.25 and (err < 1).mean() > 0.95      # informational bound


def test_kat_uniqueness_rejects_periodic_texture(oracle):
    rng = np.random.default_rng(1)
    tile = rng.integers(0, 256, (40, 8), dtype=np.uint8)
    left = np.tile(tile, (1, 20))          # period 8 along x -> near-equal minima 8 apart
    right = np.roll(left, -3, axis=1).astype(np.int32) + rng.integers(-6, 7, left.shape)
    right = np.clip(right, 0, 255).astype(np.uint8)
    base = oracle.make_params(oracle.MODE_CENSUS8, num_disparities=64, lr_check=0, subpixel=0)
    inner = slice(64, 160)
    d0 = oracle.match(base.__class__.from_buffer_copy(base), left, right)
    p = base.__class__.from_buffer_copy(base)
    fracs = []
    for u in (0, 5, 10, 20, 30):
        p.uniqueness_ratio = u
        fracs.append(float((oracle.match(p, left, right)[:, inner] != -16).mean()))
    assert fracs[0] > 0.99 and fracs[-1] < 0.3
    assert all(a >= b for a, b in zip(fracs, fracs[1:]))     # rejection grows with the ratio
    assert d0.shape == left.shape


def test_kat_lr_check_only_invalidates(oracle, synth):
    left, right, _ = synth.stereo_pair(60, 160, 0, 48, seed=21)
    right[20:40, 60:90] = right[20:40, 30:60]   # occlusion-like inconsistency
    p_off = oracle.make_params(oracle.MODE_CENSUS8, num_disparities=48, lr_check=0)
    p_on = oracle.make_params(oracle.MODE_CENSUS8, num_disparities=48, lr_check=1)
    d_off, d_on = oracle.match(p_off, left, right), oracle.match(p_on, left, right)
    changed = d_on != d_off
    assert changed.any()
    assert (d_on[changed] == -16).all()


def test_kat_speckle_sizes(oracle):
    d = np.full((30, 30), 160, np.int16)
    d[5:7, 5:7] = 800          # 4-pixel island
    d[15:25, 15:25] = 480      # 100-pixel island
    out = oracle.filter_speckles(d, -16, 50, 16)
    assert (out[5:7, 5:7] == -16).all() and (out[15:25, 15:25] == 480).all()
    assert (out[0, :] == 160).all()


def test_kat_all_invalid_when_range_exceeds_width(oracle):
    rng = np.random.default_rng(0)
    left = rng.integers(0, 256, (10, 40), dtype=np.uint8)
    for mode in (0, 1, 2):
        p = oracle.make_params(mode, min_disparity=5, num_disparities=48)
        assert (oracle.match(p, left, left) == 4 * 16).all()


def test_bad_params_rejected(oracle):
    left = np.zeros((10, 40), np.uint8)
    with pytest.raises(RuntimeError):
        oracle.match(oracle.make_params(0, num_disparities=24), left, left)


# ------------------------------------------------------------------ golden fixtures
def _golden_files():
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz"))


def test_golden_fixtures_exist():
    assert len(_golden_files()) >= 6


@pytest.mark.parametrize("name", _golden_files() if os.path.isdir(GOLDEN) else [])
def test_oracle_reproduces_golden(oracle, name):
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    p = oracle.SgmParams()
    for k, v in zip(z["param_names"], z["param_values"]):
        setattr(p, str(k), int(v))
    assert np.array_equal(oracle.match(p, z["left"], z["right"]), z["disp"])


@pytest.mark.parametrize("uniq", [0, 10])
def test_kat_all_sums_saturated_is_invalid(oracle, uniq):
    """OpenCV's `Sval < minS` from minS = MAX_COST never fires when every S equals MAX_COST:
    bestDisp stays -1 and the pixel is INVALID (and disp2 is not touched: the oracle must not
    read disp2cost one past the row there)."""
    w, minD, D = 90, -4, 48
    p = oracle.make_params(oracle.MODE_OCV_SGBM5, min_disparity=minD, num_disparities=D, uniqueness_ratio=uniq)
    width1 = oracle.effective(p, w, 3)["width1"]
    S = np.full((3, width1, D), 32767, np.uint16)
    S[1, ::3, 5] = 1000                        # some pixels have a real minimum
    disp = oracle.wta(p, S, w)
    invalid = (minD - 1) * 16
    x0 = max(minD + D, 0)
    assert (disp[0] == invalid).all() and (disp[2] == invalid).all()
    assert (disp[1, x0:x0 + width1][::3] != invalid).any()
