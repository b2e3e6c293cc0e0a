"""Synthetic rectified stereo pairs (SURVEY.md §8d "one generator, used by both CPU and GPU").

Pure numpy, deterministic from a seed (numpy PCG64):
  * left image: i.i.d. uniform u8 noise, 3x3 box blur with round-half-up, so BT / census
    costs are informative;
  * ground truth g(x, y): 4 horizontal bands, each a slanted plane a + b*x + c*y with
    values inside [minD + 2, minD + D - 3];
  * right image: R(x, y) = L(x + g(x, y), y), linearly interpolated and rounded; samples
    that fall outside the left image are filled with fresh noise from the same seed.
`integer_shift_pair` is the KAT variant with a constant integer g.
This module is shared input generation (bench + tests), not an oracle of results.
"""
import numpy as np


def _blur_noise(rng, h, w):
    n = rng.integers(0, 256, size=(h + 2, w + 2), dtype=np.int32)
    s = np.zeros((h, w), np.int32)
    for dy in range(3):
        for dx in range(3):
            s += n[dy:dy + h, dx:dx + w]
    return ((s + 4) // 9).astype(np.uint8)


def truth_field(h, w, min_disp, num_disp, seed):
    rng = np.random.default_rng(seed + 7919)
    lo, hi = min_disp + 2, min_disp + num_disp - 3
    g = np.empty((h, w), np.float64)
    ys = np.arange(h)[:, None]
    xs = np.arange(w)[None, :]
    bands = np.linspace(0, h, 5).astype(int)
    for b in range(4):
        y0, y1 = bands[b], bands[b + 1]
        a = rng.uniform(lo, hi)
        bx = rng.uniform(-0.5, 0.5) * (hi - lo) / max(w, 1)
        cy = rng.uniform(-0.5, 0.5) * (hi - lo) / max(h, 1)
        plane = a + bx * (xs - w / 2) + cy * (ys[y0:y1] - (y0 + y1) / 2)
        g[y0:y1] = np.clip(plane, lo, hi)
    return g


def stereo_pair(h, w, min_disp=0, num_disp=64, seed=0, with_truth=True):
    """Returns (left, right, truth) — u8, u8, float64 disparity in pixels (truth None if
    with_truth is False)."""
    rng = np.random.default_rng(seed)
    left = _blur_noise(rng, h, w)
    g = truth_field(h, w, min_disp, num_disp, seed)
    xs = np.arange(w)[None, :] + g
    x0 = np.floor(xs).astype(np.int64)
    fr = xs - x0
    valid = (x0 >= 0) & (x0 + 1 < w)
    x0c = np.clip(x0, 0, w - 1)
    x1c = np.clip(x0 + 1, 0, w - 1)
    rows = np.arange(h)[:, None]
    lf = left.astype(np.float64)
    samp = lf[rows, x0c] * (1 - fr) + lf[rows, x1c] * fr
    fill = _blur_noise(np.random.default_rng(seed + 104729), h, w).astype(np.float64)
    right = np.where(valid, samp, fill)
    right = np.floor(right + 0.5).clip(0, 255).astype(np.uint8)
    return left, right, (truth_left(g) if with_truth else None)


def truth_left(g_right):
    """g is defined on right-image columns (R(x') = L(x' + g(x'))); the disparity of left
    pixel x solves d = g(x - d). Fixed-point iteration (|dg/dx| < 1) with linear interp."""
    h, w = g_right.shape
    xs = np.arange(w, dtype=np.float64)[None, :].repeat(h, 0)
    rows = np.arange(h)[:, None]
    d = g_right.copy()
    for _ in range(30):
        xr = np.clip(xs - d, 0, w - 1)
        x0 = np.floor(xr).astype(np.int64)
        x1 = np.minimum(x0 + 1, w - 1)
        f = xr - x0
        d = g_right[rows, x0] * (1 - f) + g_right[rows, x1] * f
    return d


def integer_shift_pair(h, w, shift, seed=0):
    """KAT pair: R(x, y) = L(x + shift, y) exactly (fresh noise where x + shift >= w)."""
    rng = np.random.default_rng(seed)
    left = _blur_noise(rng, h, w)
    right = _blur_noise(np.random.default_rng(seed + 1), h, w)
    if shift < w:
        right[:, : w - shift] = left[:, shift:]
    return left, right


def batch(n, h, w, min_disp=0, num_disp=64, seed0=0):
    lefts, rights = [], []
    for i in range(n):
        l, r, _ = stereo_pair(h, w, min_disp, num_disp, seed0 + i)
        lefts.append(l)
        rights.append(r)
    return np.stack(lefts), np.stack(rights)
