"""Host logic of the census path launch (no GPU): the work list a fused launch dispatches
(census_sgm.hip census_path_items, exported as sgm_debug_path_items). Every block of every
requested direction of every frame appears exactly once, the up+WTA blocks (code 8: the
dir-1 column blocks, fused with the WTA) of the WTA group likewise, and the longest work
(the up+WTA chains) is dealt first. Blocks hold 16 lines (16 rows for the horizontal scans),
8 for D > 256, whose path lines are 32 lanes wide (census_sgm.hip LineCfg); up+WTA blocks
always 16."""
import ctypes

import numpy as np
import pytest



def items(pkg, W, H, D, minD, mask, slots, group, up):
    lib = pkg.load_library()
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, min_disparity=minD)
    n = lib.sgm_debug_path_items(ctypes.byref(p), W, H, mask, slots, group, up, None, 0)
    assert n >= 0
    out = np.zeros(max(n, 1), np.uint32)
    assert lib.sgm_debug_path_items(ctypes.byref(p), W, H, mask, slots, group, up,
                                     out.ctypes.data_as(ctypes.c_void_p), n) == n
    return out[:n]


def expected_blocks(W, H, D, minD, d, NL=None):
    """Blocks per direction: the row sweeps cover their lines' start columns (diagonals
    reach H - 1 columns further), the horizontal scans NL rows each."""
    NL = NL or (8 if D > 256 else 16)      # lines per row-sweep block / rows per horizontal block
    minX1, maxX1 = max(minD + D, 0), W + min(minD, 0)
    if d >= 6:
        return (H + NL - 1) // NL
    rx = {0: 0, 1: 0, 2: 1, 3: -1, 4: 1, 5: -1}[d]
    lo = minX1 - (H - 1 if rx > 0 else 0)
    hi = maxX1 + (H - 1 if rx < 0 else 0)
    return (hi - lo + NL - 1) // NL


@pytest.mark.parametrize("W,H,D,minD", [(1920, 1080, 256, 0), (1920, 1080, 128, 0), (640, 45, 48, 3),
                                        (500, 20, 400, -7), (300, 7, 16, 0)])
@pytest.mark.parametrize("group,up", [(1, 0), (2, 0), (2, 2), (3, 3), (4, 4), (2, 1)])
@pytest.mark.parametrize("slots", [256, 7])
def test_work_list_covers_every_block_once(pkg, W, H, D, minD, group, up, slots):
    it = items(pkg, W, H, D, minD, 0xFF, slots, group, up)
    code, f, lb = it >> 24, (it >> 22) & 3, it & 0x3FFFFF
    seen = set(zip(code.tolist(), f.tolist(), lb.tolist()))
    assert len(seen) == len(it)                                    # no duplicates
    want = {(d, fr, b) for d in range(8) for fr in range(group) for b in range(expected_blocks(W, H, D, minD, d))}
    want |= {(8, fr, b) for fr in range(up) for b in range(expected_blocks(W, H, D, minD, 1, NL=16))}
    assert seen == want
    n_up = int((code == 8).sum())
    if n_up:                                                       # the longest chains lead
        assert (code[:min(n_up, slots)] == 8).all()


def test_work_list_direction_mask(pkg):
    it = items(pkg, 1920, 1080, 256, 0, 0xFD, 256, 2, 2)           # the steady launch's 7 + up+WTA
    assert 1 not in set((it >> 24).tolist())
    assert {0, 2, 3, 4, 5, 6, 7, 8} == set((it >> 24).tolist())
