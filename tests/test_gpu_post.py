"""GPU parity — post filters (medianBlur 3x3, filterSpeckles) against the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(1, 1), (1, 9), (7, 1), (33, 65), (480, 640)])
def test_median3(engine, oracle, shape):
    rng = np.random.default_rng(shape[0] + 7 * shape[1])
    d = rng.integers(-2000, 5000, shape).astype(np.int16)
    assert np.array_equal(engine.median3(d), oracle.median3(d))


@pytest.mark.parametrize("max_size,max_diff", [(0, 16), (4, 0), (20, 16), (100, 64), (100000, 64)])
def test_speckles_random(engine, oracle, max_size, max_diff):
    rng = np.random.default_rng(max_size * 3 + max_diff)
    d = (rng.integers(0, 8, (120, 160)) * 16).astype(np.int16)
    d = np.repeat(np.repeat(d[::4, ::4], 4, 0), 4, 1)[:120, :160].copy()      # blocky regions
    d[rng.random(d.shape) < 0.1] = -16
    assert np.array_equal(engine.filter_speckles(d, -16, max_size, max_diff),
                          oracle.filter_speckles(d, -16, max_size, max_diff))


def test_speckles_one_giant_component(engine, oracle):
    """A single 1080p-sized component (worst case for union-find chain lengths)."""
    y, x = np.mgrid[0:1080, 0:1920]
    d = ((x + y) % 3 * 16).astype(np.int16)
    d[500:510, 900:910] = 2000
    out = engine.filter_speckles(d, -16, 100, 16)
    assert np.array_equal(out, oracle.filter_speckles(d, -16, 100, 16))
    assert (out[500:510, 900:910] == -16).all()


@pytest.mark.parametrize("shape", [(37, 101), (1, 300), (300, 1), (17, 130), (65, 64)])
def test_speckles_ragged_tiles(engine, oracle, shape):
    """Image sizes that cut the 64 x 16 union-find tiles: components crossing partial tiles."""
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    d = (rng.integers(0, 3, shape) * 16).astype(np.int16)
    d[rng.random(shape) < 0.15] = -16
    for max_size in (0, 3, 40):
        assert np.array_equal(engine.filter_speckles(d, -16, max_size, 16),
                              oracle.filter_speckles(d, -16, max_size, 16)), max_size


def test_speckles_serpentine(engine, oracle):
    """One long serpentine component winding through many tiles (border merges chained
    over the whole image), beside small isolated blobs."""
    h, w = 96, 200
    d = np.full((h, w), -16, np.int16)
    for r in range(0, h, 4):
        d[r, 1:w - 1] = 64
        c = w - 2 if (r // 4) % 2 == 0 else 1
        d[r:r + 4, c] = 64
    d[2::8, 5::9] = 400
    for max_size in (1, 500, 5000):
        assert np.array_equal(engine.filter_speckles(d, -16, max_size, 16),
                              oracle.filter_speckles(d, -16, max_size, 16)), max_size
