"""Node-shard exchange layouts at the driver's GPU counts, computed on the
host (gs_shard_plan_info, no device): with the default four pipeline parts
of RCCL no single all-to-all of configs 4 and 5 at N = 2, 4, 8 reaches the
2^30 bytes per rank past which RCCL 2.26's all_to_all_single returns wrong
bytes (ShardedNetwork refuses such a layout), and the
library's layout is the one the CPU protocol model (tests/model_sharded.py)
runs."""
import pytest

from model_sharded import part_count, part_nodes, shard_cap, shard_range, uses_codes

CONFIGS = {"cfg4": (1 << 24, 256), "cfg5": (100_000_000, 16)}


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("world", [2, 4, 8])
def test_exchanges_below_rccl_limit(engine, cfg, world):
    from safe_gossip_amd.sharded import RCCL_MAX_BYTES, plan_info
    n, R = CONFIGS[cfg]
    for rank in range(world):
        d = plan_info(n, R, world, rank, parts=4)
        assert d["max_collective_bytes"] <= RCCL_MAX_BYTES, (cfg, world, rank, d)
        # code rows at R_pad <= 16: 8 B per A row (code + target), 4 B per B
        # row, no id rows; class rows: the 2-plane code of W words
        cls = 4 * 4 * ((R + 63) // 64)
        assert (d["row_bytes"], d["row_bytes_b"]) == ((8, 4) if R <= 16 else (cls, cls))
        assert d["codes"] == (R <= 16) and (d["idrows"] == 0) == (R <= 16)


@pytest.mark.parametrize("n,R,world,parts", [
    (600, 16, 2, 1), (5000, 16, 2, 2), (1600, 8, 3, 3), (600, 40, 2, 1), (1100, 33, 2, 2), (5000, 16, 2, 4),
    (1 << 24, 256, 8, 4), (100_000_000, 16, 8, 4),
])
def test_layout_matches_protocol_model(engine, n, R, world, parts):
    from safe_gossip_amd.sharded import plan_info
    codes = uses_codes(R)
    W = (R + 63) // 64 if R >= 64 else 1
    for rank in range(world):
        d = plan_info(n, R, world, rank, parts=parts)
        lo, m, chunk = shard_range(n, world, rank)
        assert (d["lo"], d["m"], d["chunk"]) == (lo, m, chunk)
        assert d["mP"] == part_nodes(n, world, parts, codes)
        assert d["capP"] == shard_cap(n, world, W=W, parts=parts, codes=codes)
        # parts are whole blocks: a small range holds fewer than asked, never an empty one
        assert d["parts"] == part_count(n, world, parts, codes) <= parts
        assert (d["parts"] - 1) * d["mP"] < chunk <= d["parts"] * d["mP"]


def test_rccl_one_rank_default_config5(engine):
    # bench.py --sharded --config cfg5 (one RCCL rank): code rows make its
    # exchanges ~0.4-0.8 GB, within one collective per part
    from safe_gossip_amd.sharded import RCCL_MAX_BYTES, plan_info
    d = plan_info(100_000_000, 16, 1, 0, parts=4)
    assert d["max_collective_bytes"] <= RCCL_MAX_BYTES


@pytest.mark.parametrize("n,R,world,fits", [
    # class-row shards build the next round's in-lists in LDS bins of 2 K
    # nodes (gs_shard.hip edge_bin, 8 B of LDS per bin): up to 16256 bins per
    # rank; a larger rank is refused up front, by plan_info and create alike
    ((1 << 24), 256, 1, True), (16256 * 2048, 32, 1, True), (16256 * 2048 + 1, 32, 1, False),
    ((1 << 25) + 4096, 64, 1, False), (100_000_000, 32, 4, True), (100_000_000, 32, 2, False),
    # code rows (R_pad <= 16, 2P) build no in-lists ahead: no such limit
    (100_000_000, 16, 1, True),
])
def test_class_row_rank_size_limit(engine, n, R, world, fits):
    import safe_gossip_amd as sg
    from safe_gossip_amd.sharded import plan_info
    for rank in range(world):
        if fits:
            plan_info(n, R, world, rank, parts=4)
        else:
            with pytest.raises(sg.DeviceError, match="status -2"):
                plan_info(n, R, world, rank, parts=4)
