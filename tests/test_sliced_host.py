"""Host-side logic of the rumor-sliced network (no GPU): the known-set merge
places each slice's rumor bits at its offset (safe_gossip_amd/sliced.py)."""
import numpy as np
import pytest

from safe_gossip_amd.sliced import merge_known


@pytest.mark.parametrize("R,world", [(100, 3), (256, 8), (7, 3), (130, 4), (64, 2), (1, 1), (4096, 5)])
def test_merge_known_matches_bitwise_concat(R, world):
    rng = np.random.default_rng(R * 31 + world)
    n = 37
    bounds = [g * R // world for g in range(world + 1)]
    kw = (R + 63) // 64
    full = rng.integers(0, 2, size=(n, R), dtype=np.uint8)
    per = []
    for g in range(world):
        lo, hi = bounds[g], bounds[g + 1]
        bits = np.zeros((n, ((hi - lo + 63) // 64) * 64), dtype=np.uint8)
        bits[:, :hi - lo] = full[:, lo:hi]
        per.append(np.packbits(bits, axis=1, bitorder="little").view(np.uint64))
    pad = np.zeros((n, kw * 64), dtype=np.uint8)
    pad[:, :R] = full
    ref = np.packbits(pad, axis=1, bitorder="little").view(np.uint64)
    np.testing.assert_array_equal(merge_known(per, bounds, n, kw), ref)
