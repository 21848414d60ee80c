"""Host-side checks of the dropout mask stream (no GPU): the draw of element i
is the splitmix64 finaliser of seed + phi * (i + 1) (epilogue.hip drop_u,
restated in numpy here), so a slice at element offset o drawn under
seed + phi * o is the whole tensor's draw -- what ops.dropout(offset=) and
GLSTMModel's last-step-only dropout rely on."""
import numpy as np

from cnn_graph_amd.ops import DROP_WEYL

M64 = (1 << 64) - 1


def draws(seed: int, n: int) -> np.ndarray:
    """u in [0, 1) of elements 0..n-1 under seed (numpy uint64 wraps mod 2^64)."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + np.uint64(DROP_WEYL) * i
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def test_offset_folds_into_seed():
    seed, n = 0xFEEDFACECAFEBEEF, 4096
    full = draws(seed, n)
    for off in (0, 1, 7, 1000, 4095):
        folded = (seed + DROP_WEYL * off) & M64
        assert np.array_equal(draws(folded, n - off), full[off:]), off


def test_keep_rate_and_range():
    u = draws(12345, 1 << 16)
    assert u.min() >= 0.0 and u.max() < 1.0
    keep = np.float32(0.8)
    kept = np.floor(keep + u).sum()
    n = u.size
    assert abs(kept - 0.8 * n) < 6 * np.sqrt(n * 0.8 * 0.2)


def test_negative_offset_refused():
    import pytest
    from cnn_graph_amd import ops
    with pytest.raises(ValueError):
        ops.dropout(None, 0.8, 1, offset=-1)
