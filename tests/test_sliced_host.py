"""Host-side logic of the rumor-sliced network (no GPU): the known-set merge
places each slice's rumor bits at its offset, and one RPC's answers from the
slices merge into a single Gossip's (safe_gossip_amd/sliced.py)."""
import numpy as np
import pytest

from safe_gossip_amd.sliced import merge_answers, merge_known


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


def test_merge_answers(engine):
    enc = engine.rpc_encode
    empty_pull = enc(True, b"", 0)
    a, b, c = enc(True, b"\x01", 1), enc(True, b"\x02\x00", 255), enc(True, b"\x02", 2)
    # no slice answered (a Pull, or not a first Push)
    assert merge_answers([[], [], []]) == []
    # every slice answered empty: ONE empty Pull (src/gossip.rs:143-148)
    assert merge_answers([[empty_pull], [empty_pull], [empty_pull]]) == [empty_pull]
    # live entries in some slices: their frames in key (byte) order, no empty frame
    assert merge_answers([[b], [empty_pull], [a, c]]) == [a, c, b]
    assert merge_answers([[empty_pull], [c]]) == [c]
